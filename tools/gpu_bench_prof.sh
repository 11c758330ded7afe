#!/bin/bash
# bench (default args) + rocprofv3 kernel stats (data leg; cov d=1000 leg; cov d=5000 leg)
# + PMC HBM traffic passes (FETCH_SIZE, WRITE_SIZE, each its own run) for the data leg.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; grep -v amdgpu.ids gpurun_out/bench.err | tail -6
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-cov --no-fit --no-large --no-mlp > $R/gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof data stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cov -o cov --output-format csv -- python3 $R/bench.py --workload cov --cov-steps 2000 --no-cpu --no-fit --no-large > $R/gpurun_out/prof_cov.log 2>&1; rc=$?
echo "rocprof cov stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_large -o large --output-format csv -- python3 $R/bench.py --no-data --no-cov --no-fit --no-cpu --large-steps 200 > $R/gpurun_out/prof_large.log 2>&1; rc=$?
echo "rocprof large stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-cov --no-fit --no-large --no-mlp --profile-reps 1 > $R/gpurun_out/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write -o write --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-cov --no-fit --no-large --no-mlp --profile-reps 1 > $R/gpurun_out/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"
ls $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write 2>/dev/null | head
exit $rc
