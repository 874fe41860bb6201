# Round 2: parity (fail-fast) after the padded-bitmap fix and the partitioned varlen; C1/M1 bench
# lines; C3 hub sweep; M1 PMC traffic passes and rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_varlen.py tests/test_blob_abi.py "tests/test_gpu_fullsize.py::test_c1_fof_all_roots_rmat16" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAIL; grep -m3 -B2 -A25 "^____" $O/tests.log | head -60; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/dist.log 2>&1
rc=$?; tail -5 $O/dist.log
[ $rc -eq 0 ] || { echo DIST_FAIL; grep -m3 -B2 -A25 "^____" $O/dist.log | head -60; exit 1; }
timeout -k 10 300 python -u bench.py --query c1 --steps 20 --warmup 3 > $O/c1.json 2> $O/c1.err || { tail $O/c1.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/m1.json 2> $O/m1.err || { tail $O/m1.err; exit 1; }
for h in 262144 1048576 4194304; do
  OMX_PULL_HUBS=$h timeout -k 10 300 python -u bench.py --query c3 --steps 5 --warmup 2 --no-cpu-baseline > $O/c3_h$h.json 2> $O/c3_h$h.err || { tail $O/c3_h$h.err; exit 1; }
done
for f in c1 m1 c3_h262144 c3_h1048576 c3_h4194304; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:5]})"; done
bash tools/pmc.sh k_expand_heavy_sliced $O/pmc_m1 --steps 3 --warmup 1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o m1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo ALL_OK
