#!/usr/bin/env bash
# One parameterised GPU runner (replaces the round-named one-shot scripts/gpu_r*_*.sh runners).
#
#   scripts/gpu_run.sh TAG STEP [STEP ...]
#
# Runs the steps in order on the GPU box, each under its own time limit, and stops at the first
# failing step (a fault, abort, time limit or test failure ends the call: nothing more touches the
# GPU). Every step writes gpurun_out/TAG/NN_<kind>.log, whose first line is the exact command it ran.
#
# STEP forms:
#   smoke                      __graft_entry__.smoke()
#   suite                      the whole GPU test suite (pytest -m gpu)
#   tests=ARGS                 pytest ARGS (e.g. tests="tests/test_ipc_gpu.py -k world")
#   bench=ARGS                 python bench.py ARGS
#   resnet=ARGS                python bench_resnet.py ARGS
#   prof=SCRIPT ARGS           rocprofv3 --kernel-trace --stats of python SCRIPT ARGS (kernel table in the log)
#   pmc=COUNTERS;SCRIPT ARGS   one rocprofv3 --pmc pass (counters of ONE pass; no tracing domains)
#   ab=N;ENV_A|ENV_B;ARGS      N interleaved bench.py ARGS runs per arm, arm A with env ENV_A, B with ENV_B
#                              (space-separated VAR=VALUE lists; the arms alternate A B A B ...)
#   py=SCRIPT ARGS             python SCRIPT ARGS (probes under tools/)
#
# Per-step limits (seconds) come from TFD_STEP_TIMEOUT (default 900; smoke 300). While a step runs
# a heartbeat line (step, elapsed seconds, last log line) goes to stdout every 60 s.
set -u -o pipefail
TAG=${1:?usage: scripts/gpu_run.sh TAG STEP...}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
LIMIT=${TFD_STEP_TIMEOUT:-900}
N=0

run() {  # run NAME LIMIT CMD... : one step, logged, time-bounded, with a heartbeat
  local name=$1 lim=$2
  shift 2
  N=$((N + 1))
  local log
  log=$(printf '%s/%02d_%s.log' "$OUT" "$N" "$name")
  { echo "# cmd: $*"; echo "# start: $(date -Is)  limit: ${lim}s"; } > "$log"
  timeout -k 10 "$lim" "$@" >> "$log" 2>&1 &
  local pid=$! t0=$SECONDS
  while kill -0 "$pid" 2>/dev/null; do
    sleep 5
    if (( (SECONDS - t0) % 60 < 5 && SECONDS - t0 >= 60 )); then
      echo "[$TAG $N $name] running $((SECONDS - t0)) s: $(tail -c 300 "$log" | tr '\n' ' ' | tail -c 160)"
    fi
  done
  wait "$pid"
  local rc=$?
  echo "# exit: $rc after $((SECONDS - t0)) s" >> "$log"
  echo "[$TAG $N $name] exit $rc after $((SECONDS - t0)) s ($log)"
  tail -n 4 "$log"
  return $rc
}

PYTEST=(python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread)

for step in "$@"; do
  case "$step" in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    suite) run suite "${TFD_SUITE_TIMEOUT:-1150}" "${PYTEST[@]}" tests -m gpu || exit $? ;;
    tests=*) eval "args=(${step#tests=})"; run tests "$LIMIT" "${PYTEST[@]}" "${args[@]}" || exit $? ;;
    bench=*) eval "args=(${step#bench=})"; run bench "$LIMIT" python -u bench.py "${args[@]}" || exit $? ;;
    resnet=*) eval "args=(${step#resnet=})"; run resnet "$LIMIT" python -u bench_resnet.py "${args[@]}" || exit $? ;;
    py=*) eval "args=(${step#py=})"; run py "$LIMIT" python -u "${args[@]}" || exit $? ;;
    prof=*)
      eval "args=(${step#prof=})"
      d="$OUT/prof$((N + 1))"
      run prof "$LIMIT" rocprofv3 --kernel-trace --stats -d "$d" -o run -- python3 "${args[@]}" || exit $?
      python tools/prof_summary.py "$(find "$d" -name '*results.db' -print -quit)" >> "$(printf '%s/%02d_prof.log' "$OUT" "$N")" 2>&1 || true ;;
    pmc=*)
      spec=${step#pmc=}
      ctrs=${spec%%;*}
      eval "args=(${spec#*;})"
      d="$OUT/pmc$((N + 1))"
      run pmc 120 rocprofv3 --pmc $ctrs --kernel-trace -d "$d" -o run -- python3 "${args[@]}" || exit $?
      python tools/pmc_summary.py "$(find "$d" -name '*results.db' -print -quit)" >> "$(printf '%s/%02d_pmc.log' "$OUT" "$N")" 2>&1 || true ;;
    ab=*)
      spec=${step#ab=}
      reps=${spec%%;*}
      rest=${spec#*;}
      envs=${rest%%;*}
      eval "args=(${rest#*;})"
      env_a=${envs%%|*}
      env_b=${envs#*|}
      for ((i = 0; i < reps; i++)); do
        run "abA" "$LIMIT" env $env_a python -u bench.py "${args[@]}" || exit $?
        run "abB" "$LIMIT" env $env_b python -u bench.py "${args[@]}" || exit $?
      done ;;
    *) echo "unknown step: $step" >&2; exit 2 ;;
  esac
done
