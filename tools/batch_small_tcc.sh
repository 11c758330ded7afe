#!/bin/bash
# One GPU call (development): the TCC regularizer inside the persistent small loop (d <= 32):
# the TCC tier and the small-loop tier on the product library, the small-vs-graph experiment test,
# timings and the bench's tcc leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_small.py || exit $?
cp $O/gpu_tests.log $O/gpu_tests_small_tcc.log
bash tools/gpu.sh exptests tests/test_exp_paths.py::test_small_path_tcc_vs_graph_path || exit $?
timeout -k 10 300 python tools/probe_perf.py tcc > $O/tcc_small.log 2>&1 || exit $?
MIDAGMA_EXP_SMALL_TCC=0 timeout -k 10 300 python tools/probe_perf.py tcc > $O/tcc_graph.log 2>&1 || exit $?
timeout -k 10 300 python tools/probe_perf.py small > $O/small_notrek.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-data --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-logistic --no-small \
  > $O/bench_tcc.json 2> $O/bench_tcc.err || exit $?
echo batch done
