# Round 2: ridbag decode (LDS-staged rows, batched loads): parity + kernel time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r18
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ridbag.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
[ $rc -eq 0 ] || { echo TEST_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ridbag -o rb --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ridbag_bench.py --scale 22 --reps 2 > $GRAFT_REPO_ROOT/$O/ridbag.json 2> $GRAFT_REPO_ROOT/$O/ridbag.err ) || { echo PROF_FAIL; tail $O/ridbag.err; exit 1; }
cat $O/ridbag.json
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof_ridbag/rb_kernel_stats.csv')))[:3]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
echo ALL_OK
