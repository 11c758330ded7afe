#!/bin/bash
# first GPU session: layout probe, gpu tests, perf probe
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tests/probes/layout_probe.py > gpurun_out/layout.log 2>&1; rc=$?
echo "layout rc=$rc"; cat gpurun_out/layout.log | tail -5
[ $rc -ne 0 ] && exit $rc
MIDAGMA_LIB=$PWD/midagma_amd/libmidagma_hip_alt.so timeout -k 10 300 python tests/probes/layout_probe.py > gpurun_out/layout_alt.log 2>&1; rc=$?
echo "layout alt rc=$rc"; tail -5 gpurun_out/layout_alt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -rfE -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python tools/probe_perf.py all > gpurun_out/probe.log 2>&1; rc=$?
echo "probe rc=$rc"; cat gpurun_out/probe.log
exit $rc
