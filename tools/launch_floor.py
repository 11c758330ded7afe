"""Dependent-launch floor of a replayed hipGraph on this GPU (development tool):
N tiny kernels in one stream, captured once, replayed; time per kernel = the floor a chain of
dependent launches (the cov slot's ~24) pays before any work.  Also the same for kernels of
256 and 1024 workgroups that each touch one 8-byte value per thread (launch + dispatch of the
grid + drain), the shapes of the blocked inverse's series / panel launches.

    python tools/launch_floor.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def chain(n_kernels, numel, reps=50):
    x = torch.zeros(numel, dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n_kernels):
            x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * n_kernels)


if __name__ == "__main__":
    out = {}
    # torch's elementwise kernel: 4 elements per thread, 128 threads per block (unrolled)
    for label, numel in (("1_workgroup", 64), ("256_workgroups", 256 * 512), ("1024_workgroups", 1024 * 512)):
        out[label] = {str(n): round(chain(n, numel), 3) for n in (24, 96)}
    print(json.dumps({"us_per_dependent_launch_in_graph": out,
                      "device": torch.cuda.get_device_name(0)}), flush=True)
