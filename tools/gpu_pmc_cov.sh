#!/bin/bash
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE; each its own run) over the cov-mode slots at
# d=1000 and d=5000 (tools/probe_perf.py), summarized per kernel by tools/pmc_summary.py
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for w in d1000 d5000; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc_${w}_$c -o p --output-format csv -- python3 $R/tools/probe_perf.py $w > $R/gpurun_out/pmc_${w}_$c.log 2>&1; rc=$?
    echo "$w $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_${w}_FETCH_SIZE $R/gpurun_out/pmc_${w}_WRITE_SIZE $R/gpurun_out/pmc_cov_$w.json || exit 1
done
exit 0
