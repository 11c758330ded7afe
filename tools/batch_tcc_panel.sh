#!/bin/bash
# One GPU call (development): the product tier's TCC / blocked tests, then the experiments build's
# 4 x 4-block TCC kernel (MIDAGMA_EXP_TCC_BLK4) and 64 x 64 panels (MIDAGMA_EXP_PANEL64_MIN):
# parity, timings, a trace.  Every GPU step has its own time limit; the first failure ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
EXP="$R/midagma_amd/libmidagma_hip_exp.so"
T="tests/test_gpu_tcc.py tests/test_gpu_parity.py::test_full_fit_float32_dtype tests/test_gpu_parity.py::test_blocked_fast_path_trajectory tests/test_gpu_parity.py::test_large_d_split_k_score_and_trajectory tests/test_gpu_configs.py::test_config3_d5000 tests/test_gpu_configs.py::test_config3_d5000_timed_window"
bash tools/gpu.sh tests $T || exit $?
cp $O/gpu_tests.log $O/gpu_tests_product.log
MIDAGMA_LIB=$EXP MIDAGMA_EXP_TCC_BLK4=1 bash tools/gpu.sh tests tests/test_gpu_tcc.py || exit $?
cp $O/gpu_tests.log $O/gpu_tests_tcc_blk4.log
MIDAGMA_LIB=$EXP MIDAGMA_EXP_PANEL64_MIN=2048 bash tools/gpu.sh tests tests/test_gpu_parity.py::test_blocked_fast_path_trajectory \
  tests/test_gpu_parity.py::test_large_d_split_k_score_and_trajectory tests/test_gpu_configs.py::test_config3_d5000 || exit $?
cp $O/gpu_tests.log $O/gpu_tests_panel64.log
timeout -k 10 300 python tools/probe_perf.py tcc > $O/tcc_old.log 2>&1 || exit $?
MIDAGMA_EXP_TCC_BLK4=1 timeout -k 10 300 python tools/probe_perf.py tcc > $O/tcc_blk4.log 2>&1 || exit $?
MIDAGMA_EXP_TCC_BLK4=1 timeout -k 10 300 python tools/probe_perf.py tccnb > $O/tcc_nb.log 2>&1 || exit $?
(cd /tmp && MIDAGMA_EXP_TCC_BLK4=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_tcc20b -o tcc \
  --output-format csv -- python3 $R/tools/probe_perf.py tcc20 > $R/$O/prof_tcc20b.log 2>&1) || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_p32.log 2>&1 || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 MIDAGMA_EXP_PANEL64_MIN=2048 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_p64.log 2>&1 || exit $?
MIDAGMA_EXP_PANEL64_MIN=2048 MIDAGMA_EXP_P64_CHAINS=1 timeout -k 10 300 python tools/probe_perf.py large3 > $O/large3_p64c.log 2>&1 || exit $?
MIDAGMA_DEBUG_HANDBACKS=1 MIDAGMA_EXP_B2_512=1 timeout -k 10 300 python tools/probe_perf.py d5000 > $O/d5000_b512.log 2>&1 || exit $?
MIDAGMA_LIB=$EXP MIDAGMA_EXP_TCC_BLK4=1 timeout -k 10 600 python bench.py --no-data --no-fit --no-fit4 --no-cov --no-large \
  --no-mlp --no-logistic --no-small > $O/bench_tcc.json 2> $O/bench_tcc.err || exit $?
echo batch done
