#!/bin/bash
# One GPU call (round 6): the r04 / current X^T Y PMC comparison, then the TCC
# probes on the final sweep-budget rule.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/batch_pmc_r04_r05.sh > gpurun_out/pmc_r04_r05.log 2>&1 || { tail -5 gpurun_out/pmc_r04_r05.log; exit 1; }
cat gpurun_out/pmc_r04_r05.log
timeout -k 10 500 python tools/probe_perf.py tccfix 100 300 1000 > gpurun_out/probe_tccfix5.log 2>&1 || exit $?
timeout -k 10 500 python tools/probe_perf.py tccphase > gpurun_out/probe_tccphase4.log 2>&1 || exit $?
echo batch done
