#!/bin/bash
# DagmaNonlinear tests with the fused MLP tail, then config-5 timing fused vs PyTorch tail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nonlinear.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mlptail_tests.log 2>&1; rc=$?
tail -3 gpurun_out/mlptail_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_mlptail.log
echo "--- FUSED" > $L
timeout -k 10 300 python tests/probes/probe_mlp.py >> $L 2>&1 && \
echo "--- TORCH TAIL" >> $L && MIDAGMA_NO_MLP_TAIL=1 timeout -k 10 300 python tests/probes/probe_mlp.py >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L
exit $rc
