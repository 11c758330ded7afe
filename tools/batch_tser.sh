#!/bin/bash
# One GPU call (development): the next block's series inside the trailing update (gemm.hip
# trail_series_kernel, knob MIDAGMA_EXP_TRAIL_SERIES): bit-identity test, then timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh exptests tests/test_exp_paths.py::test_trail_series_bit_identical || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 MIDAGMA_EXP_TRAIL_SERIES=64 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_ts64.log 2>&1 || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 MIDAGMA_EXP_TRAIL_SERIES=32 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_ts32.log 2>&1 || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_ts0.log 2>&1 || exit $?
echo batch done
