#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tests/probes/debug_stage5.py > gpurun_out/debug5.log 2>&1; rc=$?
echo "debug rc=$rc"; tail -40 gpurun_out/debug5.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -8 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o r1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu --cov-steps 200 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof.log
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*"
exit $rc
