#!/bin/bash
# One GPU call: the X^T Y GEMM's HBM traffic on the round-4 tree
# (tools/r04_tree: its bench.py and library, built from commit 8b7d7af; git-ignored) and on this
# tree, back to back on one box, twice each (r04, cur, r04, cur): FETCH_SIZE and WRITE_SIZE passes
# (one run each) of the data leg, summarised per kernel by tools/pmc_summary.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O="$R/gpurun_out"
SKIP="--steps 5 --warmup 1 --no-cpu --no-check --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-logistic --no-small --no-tcc --profile-reps 1"
for tree in r04 cur r04b curb; do
  case $tree in
    r04*) B="$R/tools/r04_tree/bench.py $SKIP" ;;
    *) B="$R/bench.py $SKIP --no-group" ;;
  esac
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace -d "$O/pmc_${tree}_$c" -o p --output-format csv \
      -- python3 $B > "$O/pmc_${tree}_$c.log" 2>&1) || { echo "pmc $tree $c failed"; exit 1; }
  done
  python3 tools/pmc_summary.py "$O/pmc_${tree}_FETCH_SIZE" "$O/pmc_${tree}_WRITE_SIZE" "$O/pmc_$tree.json" \
    "{\"d\": 1000, \"n\": 1000000, \"world\": 1, \"tree\": \"$tree\"}" > /dev/null || exit 1
  python3 - "$O/pmc_$tree.json" "$tree" <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
for k, v in j["kernels"].items():
    if "gemm_pipe" in k:
        print(sys.argv[2], k, round(v["hbm_bytes_corrected"] / 1e9, 2), "GB per launch,", v["launches"], "launches")
PY
done
echo batch done
