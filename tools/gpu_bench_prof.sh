#!/bin/bash
# bench (default args) + rocprofv3 kernel stats + PMC HBM traffic passes for the dominant kernels
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; grep -v amdgpu.ids gpurun_out/bench.err | tail -6
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --cov-steps 300 > $R/gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-cov --profile-reps 1 > $R/gpurun_out/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write -o write --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-cov --profile-reps 1 > $R/gpurun_out/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"
ls $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write 2>/dev/null | head
exit $rc
