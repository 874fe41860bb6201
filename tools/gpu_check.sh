#!/bin/bash
# GPU-box check used during development: GPU parity tests, then C2 bench variants.
# usage: tools/gpu_check.sh [tests|notests] [bench args...]
set -o pipefail
mkdir -p gpurun_out
if [ "$1" != "notests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -5 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
shift
for hd in ${HDS:-256}; do
  OMX_HEAVY_DEG=$hd timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_hd$hd.log 2>&1 || { tail -5 gpurun_out/bench_hd$hd.log; exit 1; }
  python - gpurun_out/bench_hd$hd.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "GTEPS %.1f ms %.3f dom %s frac %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"]))
print({k: (round(v["ms_per_step"], 3), v["GBps"] and round(v["GBps"])) for k, v in list(d["kernels"].items())[:6]})
PY
done
