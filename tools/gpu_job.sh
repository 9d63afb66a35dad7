# One parametrised GPU job for gpurun (replaces the per-experiment one-off scripts):
#
#   gpurun -- 'bash tools/gpu_job.sh <job> [args...]'
#
# jobs (each GPU step under its own time limit, chained so that the first failure ends the call):
#   tests "<pytest -k expr>"   selected GPU tests              -> gpurun_out/tests.log
#   suite                      the whole -m gpu suite + smoke   -> gpurun_out/suite.log
#   ab <ab_bench.py args>      in-process A/B of model options  -> gpurun_out/ab.log
#   bench [@NAME] <bench.py args>  one bench line              -> gpurun_out/bench[_NAME].log
#   prof <round> [pmc]         tools/profile_round.sh (rocprof stats + PMC traffic + MFMA busy)
#   py <script> [args]         any repo script under a 600 s limit -> gpurun_out/py.log
# Several jobs can be chained with '+': gpu_job.sh tests "ring" + ab --layers 1 --variant attn_diag=0
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"

run_job() {
  local job=$1; shift
  case "$job" in
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$1" \
        > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; return 1; }
      grep -E "PASSED|FAILED|passed|failed" "$O/tests.log" | tail -30 ;;
    suite)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
        > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; return 1; }
      grep -E "passed|failed" "$O/suite.log" | tail -3
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -3 ;;
    ab)
      timeout -k 10 500 python3 tools/ab_bench.py "$@" > "$O/ab.log" 2>&1 || { tail -30 "$O/ab.log"; return 1; }
      grep -v amdgpu.ids "$O/ab.log" ;;
    bench)   # optional first argument @NAME: log to bench_NAME.log (several bench jobs in one call)
      local bl="$O/bench.log"
      case "$1" in @*) bl="$O/bench_${1#@}.log"; shift ;; esac
      timeout -k 10 500 python3 bench.py "$@" > "$bl" 2>&1 || { tail -30 "$bl"; return 1; }
      grep '^{' "$bl" | tail -1 ;;
    prof)
      bash "$R/tools/profile_round.sh" "$@" ;;
    py)
      timeout -k 10 600 python3 "$@" > "$O/py.log" 2>&1 || { tail -30 "$O/py.log"; return 1; }
      grep -v amdgpu.ids "$O/py.log" | tail -60 ;;
    *)
      echo "unknown job $job"; return 2 ;;
  esac
}

args=()
for a in "$@"; do
  if [ "$a" = "+" ]; then
    run_job "${args[@]}"
    args=()
  else
    args+=("$a")
  fi
done
[ ${#args[@]} -gt 0 ] && run_job "${args[@]}"
