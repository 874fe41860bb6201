# Round 2: C3 pull — hub array in degree-rank order: parity, then the size sweep (vertex order control).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/c3rank
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/varlen.log 2>&1
rc=$?; tail -2 $O/varlen.log
[ $rc -eq 0 ] || { echo VARLEN_FAIL; grep -m2 -A30 "^____" $O/varlen.log | head -50; exit 1; }
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:3]})"
}
run vertex_262144 OMX_PULL_HUB_ORDER=vertex OMX_PULL_HUBS=262144
run rank_262144 OMX_PULL_HUBS=262144
run rank_524288 OMX_PULL_HUBS=524288
run rank_1048576 OMX_PULL_HUBS=1048576
run rank_4194304 OMX_PULL_HUBS=4194304
run rank_131072 OMX_PULL_HUBS=131072
echo ALL_OK
