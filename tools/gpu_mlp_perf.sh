cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python tests/probes/probe_mlp.py --cpu > gpurun_out/probe_mlp.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/probe_mlp.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mlp -o mlp --output-format csv -- python3 $GRAFT_REPO_ROOT/tests/probes/probe_mlp.py --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/prof_mlp.log 2>&1; echo "rocprof rc=$?"
