# Round 2: dense-row light emission (k_expand_dense_rows) — parity on unfiltered paths, then A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/dense
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_traverse.py tests/test_gpu_dist.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
[ $rc -eq 0 ] || { echo TEST_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
run() {  # name, query, env...
  n=$1; q=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --query $q --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]})"
}
run m1_dense m1
run m1_mp m1 OMX_DENSE_ROWS=0
run m1_dense2 m1
run c1_dense c1
run c1_mp c1 OMX_DENSE_ROWS=0
run c2_dense c2
run c2_mp c2 OMX_DENSE_ROWS=0
run s1_dense s1
echo ALL_OK
