# Round 2: ridbag affine RID index (parity + time); M1 light-row variants of the distinct-source lists.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r21
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ridbag.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/ridbag_tests.log 2>&1 || { echo RIDBAG_FAIL; grep -m2 -A40 "^____" $O/ridbag_tests.log | head -60; exit 1; }
tail -1 $O/ridbag_tests.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ridbag -o rb --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ridbag_bench.py --scale 22 --reps 2 > $GRAFT_REPO_ROOT/$O/ridbag.json 2> $GRAFT_REPO_ROOT/$O/ridbag.err ) || { echo PROF_FAIL; tail $O/ridbag.err; exit 1; }
cat $O/ridbag.json
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof_ridbag/rb_kernel_stats.csv')))[:3]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
run() {  # name, query, env...
  n=$1; q=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --query $q --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:5]})"
}
run m1_default m1
run m1_lightmp m1 OMX_LIGHT_SLICED=0
run c2_lightmp c2 OMX_LIGHT_SLICED=0
echo ALL_OK
