#!/bin/bash
# One GPU call (development): the serial split sigmoid GEMM as the product default: the logistic
# parity and distributed tiers, then the bench's logistic legs on the product library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k logistic > $O/gpu_tests_sig.log 2>&1 || { tail -30 $O/gpu_tests_sig.log; exit 1; }
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed.py >> $O/gpu_tests_sig.log 2>&1 || { tail -30 $O/gpu_tests_sig.log; exit 1; }
grep -E "passed|failed" $O/gpu_tests_sig.log
timeout -k 10 300 python bench.py --no-data --no-cpu --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-small \
  --no-tcc > $O/sig_default.json 2> $O/sig_default.err || exit $?
echo batch done
