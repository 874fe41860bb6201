# Round 2: C3 — the pull waits only for live lanes (OMX_PULL_LIVE) and gathers non-hub masks only for
# vertices the hub in-edges left short (OMX_PULL_TWO). Varlen parity first, then the A/B lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/c3live
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), d['config'].get('rows_per_step'), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:3]})"
}
run base OMX_PULL_LIVE=0 OMX_PULL_TWO=0
run live OMX_PULL_LIVE=1 OMX_PULL_TWO=0
run two OMX_PULL_LIVE=0 OMX_PULL_TWO=1
run both OMX_PULL_LIVE=1 OMX_PULL_TWO=1
OMX_DEBUG_EXPAND=1 timeout -k 10 300 python -u bench.py --query c3 --steps 1 --warmup 0 --no-cpu-baseline > $O/dbg.json 2> $O/dbg.err || { tail $O/dbg.err; exit 1; }
grep "omx bfs" $O/dbg.err | head -5
echo ALL_OK
