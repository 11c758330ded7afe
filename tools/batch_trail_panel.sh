#!/bin/bash
# One GPU call (development): block g + 1's panel inside trailing update g (gemm.hip
# trail_panel_kernel, knob MIDAGMA_EXP_TRAIL_PANEL = panel workgroups): bit-identity test, then
# timings of the large-D slots (the fused path is taken at d = 5000, where the series runs inside).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh exptests tests/test_exp_paths.py::test_trail_panel_bit_identical || exit $?
for np in 0 256 512 1024; do
  MIDAGMA_EXP_TRAIL_PANEL=$np timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_tp$np.log 2>&1 || exit $?
done
echo batch done
