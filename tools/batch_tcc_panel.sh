#!/bin/bash
# One GPU call (development): TCC one-workgroup kernel + 64 x 64 panels (tests, timings, a trace).
# Every GPU step has its own time limit; the first failure ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_parity.py::test_full_fit_float32_dtype \
  tests/test_gpu_parity.py::test_blocked_fast_path_trajectory tests/test_gpu_parity.py::test_large_d_split_k_score_and_trajectory \
  tests/test_gpu_configs.py::test_config3_d5000 tests/test_gpu_configs.py::test_config3_d5000_timed_window || exit $?
timeout -k 10 300 python tools/probe_perf.py tcc > $O/tcc_blk4.log 2>&1 || exit $?
timeout -k 10 300 python tools/probe_perf.py tccnb > $O/tcc_nb.log 2>&1 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_tcc20b -o tcc --output-format csv \
  -- python3 $R/tools/probe_perf.py tcc20 > $R/$O/prof_tcc20b.log 2>&1) || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_p64.log 2>&1 || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 MIDAGMA_EXP_PANEL64_MIN=1000000 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_p32.log 2>&1 || exit $?
MIDAGMA_EXP_P64_CHAINS=1 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_p64c.log 2>&1 || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 MIDAGMA_EXP_B2_512=1 timeout -k 10 300 python tools/probe_perf.py d5000 > $O/d5000_b512.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-data --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-logistic --no-small \
  > $O/bench_tcc.json 2> $O/bench_tcc.err || exit $?
echo batch done
