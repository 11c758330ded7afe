#!/bin/bash
# quick loop: gpu tests + perf probe (args: pytest -k expression, probe mode)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
K="${1:-}"
MODE="${2:-all}"
if [ -n "$K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rfE -p no:cacheprovider -k "$K" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
else
  timeout -k 10 900 python -m pytest tests -m gpu -q -rfE -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
fi
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python tools/probe_perf.py $MODE > gpurun_out/probe.log 2>&1; rc=$?
echo "probe rc=$rc"; cat gpurun_out/probe.log | grep -v amdgpu.ids
exit $rc
