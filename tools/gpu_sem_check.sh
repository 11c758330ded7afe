cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -m pytest tests/test_gpu_sem.py -q -x > gpurun_out/sem_tests.log 2>&1; rc=$?; tail -5 gpurun_out/sem_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tests/probes/probe_sem.py > gpurun_out/probe_sem.log 2>&1; rc=$?; cat gpurun_out/probe_sem.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_sem -o sem --output-format csv -- python3 $GRAFT_REPO_ROOT/tests/probes/probe_sem.py --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_sem.log 2>&1; echo "rocprof rc=$?"
