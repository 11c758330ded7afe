cd $GRAFT_REPO_ROOT
for r in 1 2; do for x in 0 1; do
MIDAGMA_EXP_NM_XCD=$x timeout -k 10 240 python tools/probe_perf.py covds 300 1000 2000 > gpurun_out/nmxcd_${x}_$r.log 2>&1 || exit 1
echo "xmap=$x run $r"; grep steps gpurun_out/nmxcd_${x}_$r.log | cut -c1-80
done; done
