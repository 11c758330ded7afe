#!/bin/bash
# the two HBM-traffic PMC passes of gpu_bench_prof.sh (data leg only), each its own run
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-cov --no-fit --no-large --no-mlp --profile-reps 1 > $R/gpurun_out/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write -o write --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-cov --no-fit --no-large --no-mlp --profile-reps 1 > $R/gpurun_out/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"
exit $rc
