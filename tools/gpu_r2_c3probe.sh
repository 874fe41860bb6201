# Round 2: C3 — sparse pull levels gather non-hub masks through the frontier bitmap (OMX_PULL_PROBE:
# frontier-size fraction below which a level probes; 0 = never, 2 = always). Varlen parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/c3probe
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), d['config'].get('rows_per_step'), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]})"
}
run never OMX_PULL_PROBE=0
run default OMX_PULL_PROBE=0.1
run always OMX_PULL_PROBE=2
run never_nolive OMX_PULL_PROBE=0 OMX_PULL_LIVE=0
echo ALL_OK
