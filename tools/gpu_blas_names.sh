#!/bin/bash
# kernel names and durations of the rocBLAS dgemm calls in the GEMM micro (their Tensile configs)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_blas -o blas --output-format csv -- $R/tools/micro/gemm_micro 250112 blas > $R/gpurun_out/prof_blas.log 2>&1; rc=$?
echo "rc=$rc"; cat $R/gpurun_out/prof_blas.log | grep -v amdgpu.ids | tail -5
f=$(find $R/gpurun_out/prof_blas -name '*kernel_stats.csv' | head -1); cut -c1-400 "$f"
exit $rc
