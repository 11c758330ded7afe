#!/bin/bash
# One GPU call (development): the next block's series inside the trailing update (gemm.hip
# trail_series_kernel, knobs MIDAGMA_EXP_TRAIL_SERIES = workers, MIDAGMA_EXP_TS_WOFF = placement):
# bit-identity test, then timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh exptests tests/test_exp_paths.py::test_trail_series_bit_identical || exit $?
timeout -k 10 300 python tools/probe_perf.py d1000 > $O/d1000_rowpart_wt.log 2>&1 || exit $?
timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_ts0.log 2>&1 || exit $?
for w in 64 128 256; do
  for o in 1 0; do
    MIDAGMA_EXP_TRAIL_SERIES=$w MIDAGMA_EXP_TS_WOFF=$o timeout -k 10 300 python tools/probe_perf.py large3 \
      > $O/large3_ts${w}_o$o.log 2>&1 || exit $?
  done
done
echo batch done
