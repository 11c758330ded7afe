#!/bin/bash
# One GPU call (development): the single-buffered panel at a fixed prefetch depth (blockinv.hip
# binv_panel_kernel<SBPF>, knob MIDAGMA_EXP_PANEL_SB = 1..3): bit-identity test, then timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh exptests tests/test_exp_paths.py::test_panel_single_buffered_bit_identical || exit $?
for pf in 0 1 2 3; do
  MIDAGMA_EXP_PANEL_SB=$pf timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_psb$pf.log 2>&1 || exit $?
  MIDAGMA_EXP_PANEL_SB=$pf timeout -k 10 300 python tools/probe_perf.py d1000 > $O/d1000_psb$pf.log 2>&1 || exit $?
done
echo batch done
