#!/bin/bash
# the default bench line (as the driver runs it)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; grep -v amdgpu.ids gpurun_out/bench.err | tail -8
exit $rc
