# Round 2: parity of the new device features (documents, optional nodes, multi items) and the
# partitioned/varlen suites, then M1 and C2 bench lines (C2 at two heavy-row cuts).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/feat
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_varlen.py tests/test_gpu_dist.py tests/test_gpu_triangle.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/feat/tests.log 2>&1
rc=$?
tail -30 gpurun_out/feat/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAIL rc=$rc; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/feat/m1.json 2> gpurun_out/feat/m1.err || { tail gpurun_out/feat/m1.err; exit 1; }
for hd in 256 512; do
  OMX_HEAVY_DEG=$hd timeout -k 10 300 python -u bench.py --query c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/feat/c2_hd$hd.json 2> gpurun_out/feat/c2_hd$hd.err || exit 1
done
for f in m1 c2_hd256 c2_hd512; do python -c "import json;d=json.load(open('gpurun_out/feat/$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in d['kernels'].items()})"; done
