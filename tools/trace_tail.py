"""Per-kernel totals over the last `frac` of a rocprofv3 kernel trace (by dispatch start time):
the later part of a probe whose earlier part is warm-up.

    python tools/trace_tail.py gpurun_out/prof_x/p_kernel_trace.csv 0.2 [steps]
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    path, frac = sys.argv[1], float(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t_end = int(rows[-1]["End_Timestamp"])
    t_begin = int(rows[0]["Start_Timestamp"])
    cut = t_end - frac * (t_end - t_begin)
    tail = [r for r in rows if int(r["Start_Timestamp"]) >= cut]
    agg, cnt = defaultdict(float), defaultdict(int)
    for r in tail:
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
        agg[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[name] += 1
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    busy = sum(agg.values())
    print(f"last {frac:.0%}: {len(tail)} dispatches, span {span:.0f} us, kernel time {busy:.0f} us")
    for k in sorted(agg, key=agg.get, reverse=True)[:25]:
        per = f" {agg[k] / steps:8.1f} us/step {cnt[k] / steps:6.1f}/step" if steps else ""
        print(f"{k[:80]:80s} {cnt[k]:7d} {agg[k] / cnt[k]:8.2f} us{per}")


if __name__ == "__main__":
    main()
