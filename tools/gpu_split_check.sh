#!/bin/bash
# cov GEMM split-K at large d: parity subset, then d=2000 / d=5000 timings per split
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "large or blocked or d1000" > gpurun_out/split_tests.log 2>&1; rc=$?
tail -3 gpurun_out/split_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_split.log
echo "--- AUTO" > $L
timeout -k 10 300 python tools/probe_perf.py d2000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 || exit 1
for sp in 1 2 4; do
  echo "--- SPLIT $sp" >> $L
  MIDAGMA_EXP_COV_SPLIT=$sp timeout -k 10 300 python tools/probe_perf.py d2000 >> $L 2>&1 && \
  MIDAGMA_EXP_COV_SPLIT=$sp timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 || exit 1
done
grep -a -v amdgpu.ids $L | cut -c1-140
