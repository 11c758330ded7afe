#!/bin/bash
# data-mode GEMM shapes: library kernel vs rocBLAS, then one SQ PMC pass over both kernels
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 ./tools/micro/gemm_micro ${N:-1000064} ${WHICH:-xw xty blas} > gpurun_out/gemm_micro.log 2>&1; rc=$?
echo "micro rc=$rc"; cat gpurun_out/gemm_micro.log
[ $rc -ne 0 ] && exit $rc
[ -n "$NOPMC" ] && exit 0
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $R/gpurun_out/pmc_gemm -o sq --output-format csv -- $R/tools/micro/gemm_micro 250112 ${PMCWHICH:-xw xty} > $R/gpurun_out/pmc_gemm.log 2>&1; rc=$?
echo "pmc rc=$rc"
python3 $R/tools/pmc_counters.py $R/gpurun_out/pmc_gemm
exit $rc
