#!/bin/bash
# The one GPU-box driver (run under gpurun from the repo root):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu.sh TASK [ARGS...]'
# Every GPU step runs under its own `timeout -k 10`; the first failure ends the call.
#
# TASK
#   tests [PATHS/ARGS]    pytest -m gpu (default path: tests) (one process, as the driver runs it) -> gpurun_out/gpu_tests.log
#   exptests [ARGS]       pytest -m experiment on the experiments build (libmidagma_hip_exp.so, knobs.h)
#                         -> gpurun_out/exp_tests.log
#   smoke                 __graft_entry__.smoke()
#   bench [BENCH ARGS]    python bench.py -> gpurun_out/bench.json (+ .err)
#   rehearse2             bench.py --gpus 2 with both ranks on cuda:0 over gloo (the N > 1 path end to end on
#                         a one-GPU box; not a scaling number) -> gpurun_out/rehearse2.json
#   prof LEG              rocprofv3 --kernel-trace --stats of one bench leg -> gpurun_out/prof_LEG/
#                         LEG: data | cov | large | small | logistic | mlp | fit4 | tcc (one bench leg each)
#   pmc LEG               FETCH_SIZE and WRITE_SIZE passes (each its own run) of one leg,
#                         summarised per kernel -> gpurun_out/pmc_LEG.json (tools/pmc_summary.py)
#   probe NAME [ARGS]     python tools/NAME.py ARGS (probe_perf, peak_probe, blocked_debug, ...); probe_perf
#                         loads the experiments build (its comparisons set MIDAGMA_EXP_* knobs)
# Several tasks may be chained in one call: `bash tools/gpu.sh tests -- bench -- prof cov`.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp

leg_args() {
  local skip="--no-cpu --no-check --no-fit --no-fit4 --no-cov --no-large --no-mlp --no-logistic --no-small --no-tcc --no-group"
  case "$1" in
    data)     echo "--steps 5 --warmup 1 ${skip}" ;;
    cov)      echo "--workload cov --cov-steps 2000 --no-cpu --no-check --no-fit --no-fit4 --no-large" ;;
    fit4)     echo "--steps 2 --warmup 1 ${skip/--no-fit4/}" ;;
    large)    echo "--no-data ${skip/--no-large/} --large-steps 200" ;;
    mlp)      echo "--no-data ${skip/--no-mlp/}" ;;
    logistic) echo "--no-data ${skip/--no-logistic/}" ;;
    small)    echo "--no-data ${skip/--no-small/}" ;;
    tcc)      echo "--no-data ${skip/--no-tcc/}" ;;
    *) return 1 ;;
  esac
}

# workload tag bench.py matches when it reads the committed PMC summary (data leg only)
pmc_workload() {
  case "$1" in
    data) echo '{"d": 1000, "n": 1000000, "world": 1, "command": "tools/gpu.sh pmc data"}' ;;
    *) echo '{"leg": "'"$1"'"}' ;;
  esac
}

run_task() {
  local task=$1; shift
  case "$task" in
    tests)
      [ $# -eq 0 ] && set -- tests
      timeout -k 10 1500 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
        > gpurun_out/gpu_tests.log 2>&1; local rc=$?
      grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3; return $rc ;;
    exptests)
      [ $# -eq 0 ] && set -- tests
      MIDAGMA_LIB="$R/midagma_amd/libmidagma_hip_exp.so" timeout -k 10 900 python -u -m pytest -m experiment -x -v \
        --timeout 300 --timeout-method thread "$@" > gpurun_out/exp_tests.log 2>&1; local rc=$?
      grep -E "passed|failed|error" gpurun_out/exp_tests.log | tail -3; return $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; local rc=$?
      tail -3 gpurun_out/smoke.log; return $rc ;;
    bench)
      timeout -k 10 1100 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err; local rc=$?
      echo "bench rc=$rc"; cat gpurun_out/bench.json; grep -v amdgpu.ids gpurun_out/bench.err | tail -8; return $rc ;;
    rehearse2)
      MIDAGMA_BENCH_SAME_DEVICE=1 MIDAGMA_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 \
        --steps 10 --warmup 2 "$@" > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err; local rc=$?
      echo "rehearse2 rc=$rc"; cat gpurun_out/rehearse2.json; grep -v amdgpu.ids gpurun_out/rehearse2.err | tail -8
      return $rc ;;
    prof)
      local leg=$1 a
      a="$R/bench.py $(leg_args "$leg")" || return 2
      (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$leg" -o "$leg" \
        --output-format csv -- python3 $a > "$R/gpurun_out/prof_$leg.log" 2>&1); local rc=$?
      echo "prof $leg rc=$rc"; return $rc ;;
    pmc)
      local leg=$1 a c
      a="$R/bench.py $(leg_args "$leg") --profile-reps 1" || return 2
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -s KILL 600 rocprofv3 --pmc $c --kernel-trace -d "$R/gpurun_out/pmc_${leg}_$c" -o p \
          --output-format csv -- python3 $a > "$R/gpurun_out/pmc_${leg}_$c.log" 2>&1) || { echo "pmc $leg $c failed"; return 1; }
      done
      python3 tools/pmc_summary.py "gpurun_out/pmc_${leg}_FETCH_SIZE" "gpurun_out/pmc_${leg}_WRITE_SIZE" \
        "gpurun_out/pmc_$leg.json" "$(pmc_workload "$leg")"; return $? ;;
    probe)
      local name=$1; shift
      timeout -k 10 900 python "tools/$name.py" "$@" > "gpurun_out/probe_$name.log" 2>&1; local rc=$?
      tail -30 "gpurun_out/probe_$name.log"; return $rc ;;
    *) echo "unknown task $task"; return 2 ;;
  esac
}

# split the argument list on "--" into tasks
args=("$@")
cur=()
for a in "${args[@]}" "--"; do
  if [ "$a" = "--" ]; then
    if [ ${#cur[@]} -gt 0 ]; then
      run_task "${cur[@]}" || exit $?
    fi
    cur=()
  else
    cur+=("$a")
  fi
done
exit 0
