#!/bin/bash
# One GPU call (round 6): the X^T Y GEMM's fetched bytes against Y's placement (experiments build,
# MIDAGMA_EXP_Y_OFFSET bytes into its allocation; or PMC_VAR / PMC_VALS, e.g. MIDAGMA_EXP_PREPAD_MB):
# FETCH_SIZE passes of the data leg, one run each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O="$R/gpurun_out"
SKIP="--steps 5 --warmup 1 --no-cpu --no-check --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-logistic --no-small --no-tcc --no-group --profile-reps 1"
VAR=${PMC_VAR:-MIDAGMA_EXP_Y_OFFSET}
VALS=${PMC_VALS:-0 512 2048 8192 32768 0}
for off in $VALS; do
  (cd /tmp && export MIDAGMA_LIB="$R/midagma_amd/libmidagma_hip_exp.so" && export "$VAR=$off" && timeout -s KILL 300 \
    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmcy_$off" -o p --output-format csv \
    -- python3 "$R/bench.py" $SKIP > "$O/pmcy_$off.log" 2>&1) || { echo "pmc offset $off failed"; exit 1; }
  python3 - "$O/pmcy_$off" "$off" "$VAR" <<'PY'
import sys
sys.path.insert(0, "tools")
from pmc_summary import load
f, n = load(sys.argv[1], "FETCH_SIZE")
for k, v in sorted(f.items()):
    if "gemm_pipe" in k:
        print(sys.argv[3], sys.argv[2], k, round(2 * v * 1024 / 1e9, 2), "GB fetched per launch,", n[k], "launches")
PY
  rm -rf "$O/pmcy_$off"
done
echo batch done
