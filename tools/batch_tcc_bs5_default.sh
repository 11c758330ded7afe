#!/bin/bash
# One GPU call (development): the one-wave 5 x 5 TCC body as the product default for d <= 20:
# the TCC and small tiers, then the bench's TCC leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_small.py || exit $?
cp $O/gpu_tests.log $O/gpu_tests_tcc_bs5_default.log
timeout -k 10 600 python bench.py --no-data --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-logistic --no-small \
  > $O/bench_tcc.json 2> $O/bench_tcc.err || exit $?
echo batch done
