#!/bin/bash
# cov d=1000: fit wall-clock and hand-backs with 4 vs 3 product-form passes; cov split-K 2/4/8
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/probe_nm.log
export MIDAGMA_DEBUG_HANDBACKS=1
timeout -k 10 300 python tools/probe_perf.py fit > $L 2>&1 && \
echo "--- NM_PASSES=3" >> $L && MIDAGMA_EXP_NM_PASSES=3 timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1 && \
for sp in 2 4 8; do echo "--- COV_SPLIT=$sp" >> $L; MIDAGMA_EXP_COV_SPLIT=$sp timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 || exit 1; done
rc=$?
grep -v amdgpu.ids $L | awk '/drive_blocked/{n++; s+=$NF=="hand-backs"?0:0; split($0,a," "); hb+=a[4]; sl+=a[2]; next} {print} END{print "drive_blocked calls", n, "slots", sl, "hand-backs", hb}' | cut -c1-250
grep "drive_blocked" $L | awk '{hb+=$4} END{print "total hand-backs (all runs)", hb}'
exit $rc
