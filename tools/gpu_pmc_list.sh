#!/bin/bash
# list the SQ / TCC counters rocprofv3 offers on this box (for PMC pass design)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
grep -o "SQ_[A-Z0-9_]*\|TCC_[A-Z0-9_]*\|TCP_[A-Z0-9_]*" $GRAFT_REPO_ROOT/gpurun_out/counters.txt | sort -u > $GRAFT_REPO_ROOT/gpurun_out/counter_names.txt
wc -l $GRAFT_REPO_ROOT/gpurun_out/counter_names.txt
