# Round 2: C3 pull with hub-first row order (OMX_PULL_SORT): varlen parity, then C3 with and without.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r20
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/varlen.log 2>&1
rc=$?; tail -1 $O/varlen.log
[ $rc -eq 0 ] || { echo VARLEN_FAIL; grep -m2 -A30 "^____" $O/varlen.log | head -50; exit 1; }
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:3]})"
}
run sorted
run unsorted OMX_PULL_SORT=0
run sorted_h18 OMX_PULL_HUBS=262144
echo ALL_OK
