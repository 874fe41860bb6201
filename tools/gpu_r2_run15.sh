# Round 2: ridbag decoder rewrite (parity + kernel time), TRAVERSE / SELECT expand bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r15
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ridbag.py tests/test_gpu_traverse.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { echo TEST_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ridbag -o rb --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ridbag_bench.py --scale 22 --reps 2 > $GRAFT_REPO_ROOT/$O/ridbag.json 2> $GRAFT_REPO_ROOT/$O/ridbag.err ) || { echo PROF_FAIL; tail $O/ridbag.err; exit 1; }
cat $O/ridbag.json
for q in t1 s1; do
  timeout -k 10 400 python -u bench.py --query $q --steps 5 --warmup 2 --cpu-seconds 8 > $O/$q.json 2> $O/$q.err || { tail $O/$q.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$q.json'));print('$q', round(d['value'],1), round(d['ms_per_step'],3), d['config']['rows_per_step'], d['roofline']['kernel'], round(d['roofline']['frac'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:5]}, d['cpu_baseline']['value'])"
done
echo ALL_OK
