#!/bin/bash
# One GPU-box pass: GPU parity tests, the default bench line (with the CPU baseline), and the
# rocprofv3 kernel-trace summary of the same bench command.
# usage: tools/full_check.sh <outdir> [tests|notests] [bench args...]
set -o pipefail
OUT=$1; shift
MODE=$1; shift
mkdir -p "$OUT"
if [ "$MODE" != "notests" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -20 "$OUT/gpu_tests.log"; exit 1; }
  tail -1 "$OUT/gpu_tests.log"
fi
timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
tail -1 "$OUT/prof_bench.log"
find "$OUT/prof" -name '*kernel_stats.csv' -exec head -12 {} \;
