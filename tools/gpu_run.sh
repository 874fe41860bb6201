#!/bin/bash
# One parameterised GPU runner for gpurun (replaces the per-experiment scripts of rounds 1-2).
#
#   tools/gpu_run.sh <outdir under gpurun_out/> <step> [<step> ...]
#
# Steps run in order; the first failure ends the run (no further GPU work after a fault, a time limit or
# a crash). Every GPU step has its own time limit.
#   tests:<pytest args, comma-separated>       e.g. tests:tests/test_gpu_gen.py  or  tests:tests,-k,c5+or+m1
#   bench:<name>:<query>[:<bench args, comma-separated>][:ENV=V,ENV=V]
#   prof:<name>:<query>[:<bench args>][:ENV=V]  rocprofv3 --kernel-trace --stats of a short bench run
#   pmc:<name>:<query>:<timer name>:<kernel regex>[:<bench args>]  FETCH_SIZE / WRITE_SIZE / SQ passes
#                                              (tools/pmc.sh), per-launch traffic → profiles/traffic.json
#   smoke                                      __graft_entry__.smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out/$1
shift
mkdir -p "$O"
commas() { echo "$1" | tr ',' ' '; }
for step in "$@"; do
  IFS=':' read -r kind a b c d e <<< "$step"
  case "$kind" in
    tests)
      log=$O/tests_$(echo "$a" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40).log
      IFS=',' read -ra targs <<< "$a"
      targs=("${targs[@]//+/ }")  # '+' inside an argument stands for a space (-k,a+or+b)
      timeout -k 10 1100 python -u -m pytest "${targs[@]}" -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$log" 2>&1
      rc=$?
      tail -4 "$log"
      [ $rc -eq 0 ] || { echo "TESTS_FAIL rc=$rc"; grep -m3 -A30 "^____" "$log" | head -80; exit 1; }
      ;;
    bench)
      env $(commas "$d") timeout -k 10 600 python -u bench.py --query "$b" $(commas "$c") > "$O/$a.json" 2> "$O/$a.err"
      rc=$?
      [ $rc -eq 0 ] || { echo "BENCH_FAIL $a rc=$rc"; tail -20 "$O/$a.err"; exit 1; }
      python3 tools/summarize.py "$O/$a.json"
      ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && env $(commas "$d") timeout -k 10 600 rocprofv3 --kernel-trace --stats \
          -d "$GRAFT_REPO_ROOT/$O/prof_$a" -o "$a" --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --query "$b" \
          --no-cpu-baseline $(commas "$c") > "$GRAFT_REPO_ROOT/$O/prof_$a.json" 2> "$GRAFT_REPO_ROOT/$O/prof_$a.err" )
      rc=$?
      [ $rc -eq 0 ] || { echo "PROF_FAIL $a rc=$rc"; tail -20 "$O/prof_$a.err"; exit 1; }
      python3 tools/summarize.py "$O/prof_$a.json" "$O/prof_$a"
      ;;
    pmc)
      bash tools/pmc.sh "$d" "$O/pmc_$a" --query "$b" $(commas "$e") || { echo "PMC_FAIL $a"; exit 1; }
      python3 tools/pmc_traffic.py "$O/pmc_$a" "$d" "$c" "$b" --out "$O/traffic.json" || exit 1
      ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo SMOKE_FAIL; tail "$O/smoke.log"; exit 1; }
      tail -2 "$O/smoke.log"
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo GPU_RUN_OK
