#!/bin/bash
# SQ counters (one pass, no trace domains) for the data-mode GEMMs at a small n
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS --kernel-trace -d $R/gpurun_out/pmc_sq -o sq --output-format csv -- python3 $R/tools/probe_perf.py data250 > $R/gpurun_out/pmc_sq.log 2>&1; rc=$?
echo "pmc sq rc=$rc"
exit $rc
