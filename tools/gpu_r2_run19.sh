# Round 2: factorized expansion with bitmap-listed distinct sources: parity, dist, M1 / C2 lines + trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r19
mkdir -p $O
for f in parity dist fullsize; do
  timeout -k 10 500 python -u -m pytest tests/test_gpu_$f.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/$f.log 2>&1
  rc=$?; tail -1 $O/$f.log
  [ $rc -eq 0 ] || { echo FAIL $f; grep -m2 -A40 "^____" $O/$f.log | head -60; exit 1; }
done
OMX_DEBUG_EXPAND=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/m1.json 2> $O/m1.err || { tail $O/m1.err; exit 1; }
timeout -k 10 300 python -u bench.py --query c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
for f in m1 c2; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['kernel'], round(d['roofline']['frac'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:5]})"; done
grep -m4 "factorized\|omx expand" $O/m1.err
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_m1 -o m1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_m1.json 2> $GRAFT_REPO_ROOT/$O/prof_m1.err ) || { echo PROF_FAIL; tail $O/prof_m1.err; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ridbag.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/ridbag_tests.log 2>&1 || { echo RIDBAG_FAIL; grep -m2 -A40 "^____" $O/ridbag_tests.log | head -60; exit 1; }
tail -1 $O/ridbag_tests.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ridbag -o rb --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ridbag_bench.py --scale 22 --reps 2 > $GRAFT_REPO_ROOT/$O/ridbag.json 2> $GRAFT_REPO_ROOT/$O/ridbag.err ) || { echo PROF_FAIL; tail $O/ridbag.err; exit 1; }
cat $O/ridbag.json
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof_ridbag/rb_kernel_stats.csv')))[:3]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
echo ALL_OK
