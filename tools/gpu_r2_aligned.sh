# Round 2: aligned dense stores (k_expand_heavy_dense) — parity on the unfiltered paths, then M1 / C1 / C2 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/aligned
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
[ $rc -eq 0 ] || { echo TEST_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
run() {  # name, query, env...
  n=$1; q=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --query $q --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]})"
}
run m1_aligned m1
run m1_strided m1 OMX_ALIGNED_DENSE=0
run m1_aligned2 m1
run c1_aligned c1
run c1_strided c1 OMX_ALIGNED_DENSE=0
run c2_aligned c2
echo ALL_OK
