#!/bin/bash
# One GPU call (development): the logistic sigmoid GEMM in two serial K halves (gemm.hip, knob
# MIDAGMA_EXP_SIG_SPLIT): the score test, then the logistic n = 1e4 leg with and without it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh exptests tests/test_exp_paths.py::test_sigmoid_serial_split_score || exit $?
for k in 0 1 0 1; do
  MIDAGMA_LIB="$R/midagma_amd/libmidagma_hip_exp.so" MIDAGMA_EXP_SIG_SPLIT=$k timeout -k 10 300 python bench.py \
    --no-data --no-cpu --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-small --no-tcc \
    >> $O/sig_split_$k.json 2>> $O/sig_split_$k.err || exit $?
done
echo batch done
