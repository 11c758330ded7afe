#!/bin/bash
# run-to-run spread of the default bench line: two more full runs on one box
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 500 python -u bench.py > gpurun_out/bench_rep$i.log 2>&1 || exit $?
  grep -a '^{"metric"' gpurun_out/bench_rep$i.log > gpurun_out/bench_rep$i.json || exit 1
done
python - <<'PY'
import json
for i in (1, 2):
    b = json.load(open(f"gpurun_out/bench_rep{i}.json"))
    print(i, round(b["value"], 3), round(b["roofline"]["frac"], 4), round(b["cov_mode"]["value"], 1),
          round(b["config3"]["value"], 2), round(b["full_fit"]["wall_s"], 2), round(b["config5"]["value"], 1))
PY
