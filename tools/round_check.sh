#!/bin/bash
# Round-end GPU pass: every GPU parity test, the default bench line (C2, with the CPU baseline), C3/C4
# bench lines, and rocprofv3 kernel-trace summaries of the C2 and C3 bench commands.
# usage: tools/round_check.sh <outdir>
set -o pipefail
OUT=$1
mkdir -p "$OUT"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json.log" 2>&1 || { tail -20 "$OUT/bench_c2.json.log"; exit 1; }
for q in c3 c4; do
  timeout -k 10 300 python -u bench.py --query $q > "$OUT/bench_$q.json.log" 2>&1 || { tail -20 "$OUT/bench_$q.json.log"; exit 1; }
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
for q in c2 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$q" -o run --output-format csv \
    -- python3 bench.py --query $q --no-cpu-baseline > "$OUT/prof_$q.log" 2>&1 || { tail -20 "$OUT/prof_$q.log"; exit 1; }
done
for f in "$OUT"/bench_*.json.log; do tail -1 "$f" | cut -c1-400; done
