cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python tools/probe_perf.py tcc > gpurun_out/probe_tcc.log 2>&1; rc=$?; cat gpurun_out/probe_tcc.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tcc -o tcc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_perf.py tcc > $GRAFT_REPO_ROOT/gpurun_out/prof_tcc.log 2>&1; echo "rocprof rc=$?"
