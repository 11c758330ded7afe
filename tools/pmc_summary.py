"""Summarize rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) per kernel into a JSON file.

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write out.json [workload-json]

Bytes per launch follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced stream, so the
corrected fetch is 2 x FETCH_SIZE; Infinity-Cache hits are counted in FETCH_SIZE.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        if "gemm" in name:  # one template serves several GEMM shapes: key by grid as well
            name += f" grid={int(r['Grid_Size']) // int(r['Workgroup_Size'])}"
        agg[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    fetch, nf = load(sys.argv[1], "FETCH_SIZE")
    write, nw = load(sys.argv[2], "WRITE_SIZE")
    out = {"note": "per-launch averages; bytes = KiB * 1024; fetch_corrected = 2 * FETCH_SIZE (gfx950 wide reads)",
           "kernels": {}}
    if len(sys.argv) > 4:
        out["workload"] = json.loads(sys.argv[4])
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("midagma"):
            continue
        f = fetch.get(k, 0.0) * 1024
        w = write.get(k, 0.0) * 1024
        out["kernels"][k] = {"launches": nf.get(k, 0), "fetch_bytes_raw": f, "fetch_bytes_corrected": 2 * f,
                             "write_bytes": w, "hbm_bytes_corrected": 2 * f + w}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1)[:2000])


if __name__ == "__main__":
    main()
