# fused MLP fc1 + tail: GPU tests, A/B probe, kernel profile (development script)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nonlinear.py > gpurun_out/nl.log 2>&1 || { tail -30 gpurun_out/nl.log; exit 1; }
tail -1 gpurun_out/nl.log
timeout -k 10 300 python tools/probe_mlp.py 2000 fused || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mlpf -o mlpf --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_mlp.py 1000 fast > $GRAFT_REPO_ROOT/gpurun_out/prof_mlpf.log 2>&1 || exit 1
python3 - <<'PY'
import csv, os
rows=list(csv.DictReader(open(os.environ["GRAFT_REPO_ROOT"]+"/gpurun_out/prof_mlpf/mlpf_kernel_stats.csv")))
for r in rows[:16]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1000:7.2f}us")
PY
