"""Per-kernel averages of every counter in a rocprofv3 --pmc output directory (development tool).

    python tools/pmc_counters.py gpurun_out/pmc_gemm
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:60]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "SQ_BUSY_CYCLES" in cs:
            m = sum(cs["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(cs["SQ_VALU_MFMA_BUSY_CYCLES"])
            b = sum(cs["SQ_BUSY_CYCLES"]) / len(cs["SQ_BUSY_CYCLES"])
            print(f"    MFMA busy / (SQ busy * 4 SIMD * 256 CU... see guide) raw ratio {m / b:.3f}")


if __name__ == "__main__":
    main()
