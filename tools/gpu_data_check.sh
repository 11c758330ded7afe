cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q -x -k "data or logistic or distributed" > gpurun_out/xt_tests.log 2>&1; rc=$?; tail -5 gpurun_out/xt_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu --no-cov --no-fit --no-large > gpurun_out/xt_bench.json 2> gpurun_out/xt_bench.err; rc=$?; cat gpurun_out/xt_bench.json; exit $rc
