#!/bin/bash
# full GPU tests, then cov timings at d=2000 and d=5000 and the d=5000 score GEMM's L2-miss
# traffic (grouped 8 x 8 tile order per XCD in gemm_pipe_kernel)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/grp_tests.log 2>&1; rc=$?
tail -3 gpurun_out/grp_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_grp.log
timeout -k 10 300 python tools/probe_perf.py d2000 > $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1; rc=$?
grep -a "steps/s" $L | cut -c1-300
[ $rc -ne 0 ] && exit $rc
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmcg_FETCH_SIZE -o p --output-format csv -- python3 $R/tools/probe_perf.py d5000 > $R/gpurun_out/pmcg_f.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmcg_WRITE_SIZE -o p --output-format csv -- python3 $R/tools/probe_perf.py d5000 > $R/gpurun_out/pmcg_w.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcg_FETCH_SIZE $R/gpurun_out/pmcg_WRITE_SIZE $R/gpurun_out/pmc_cov_d5000_grouped.json > /dev/null
