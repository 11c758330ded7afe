#!/bin/bash
# One GPU call (development): the TCC body generalised to BS x BS blocks; the one-wave 5 x 5 form
# for d <= 20 in the small loop (knob MIDAGMA_EXP_TCC_BS5).  The TCC and small tiers on the
# product library (BS = 4 codegen changed), the experiment tests, timings with and without BS5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_small.py || exit $?
cp $O/gpu_tests.log $O/gpu_tests_tcc_bs.log
bash tools/gpu.sh exptests tests/test_exp_paths.py -k "small_path_tcc" || exit $?
for k in 0 1 0 1; do
  MIDAGMA_EXP_TCC_BS5=$k timeout -k 10 300 python tools/probe_perf.py tcc20 >> $O/tcc_bs5_$k.log 2>&1 || exit $?
done
echo batch done
