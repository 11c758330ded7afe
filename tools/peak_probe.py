"""Measured peaks of this MI355X (P and BW by microbenchmark beside the spec):
HBM bandwidth from a large device-to-device copy (read + write bytes) and FP64 matrix
throughput from a large rocBLAS DGEMM (torch.mm).  Prints one JSON line.

    python tools/peak_probe.py
"""
import json
import time

import torch


def timed(f, reps):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 30  # 8 GiB of float64
    a = torch.empty(n, dtype=torch.float64, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    t = timed(lambda: b.copy_(a), 10)
    hbm = 2 * 8 * n / t / 1e9
    del a, b
    m = 8192
    x = torch.randn(m, m, dtype=torch.float64, device=dev)
    y = torch.randn(m, m, dtype=torch.float64, device=dev)
    t = timed(lambda: torch.mm(x, y), 5)
    tf = 2 * m ** 3 / t / 1e12
    print(json.dumps({"hbm_copy_GB_per_s": hbm, "hbm_spec_GB_per_s": 8000.0, "dgemm_8192_TFLOPs": tf,
                      "fp64_matrix_spec_TFLOPs": 78.6, "device": torch.cuda.get_device_name(0)}), flush=True)


if __name__ == "__main__":
    main()
