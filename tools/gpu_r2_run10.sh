# Round 2: ridbag ingest parity; M1 kernel-trace summary + PMC traffic of its dominant kernel; C3 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ridbag.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/ridbag.log 2>&1
rc=$?; tail -3 $O/ridbag.log
[ $rc -eq 0 ] || { echo RIDBAG_FAIL; grep -m2 -A40 "^____" $O/ridbag.log | head -60; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_m1 -o m1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_m1.json 2> $GRAFT_REPO_ROOT/$O/prof_m1.err ) || { echo PROF_FAIL; tail $O/prof_m1.err; exit 1; }
bash tools/pmc.sh "k_expand_heavy<" $O/pmc_m1 --query m1 --steps 2 --warmup 1 || exit 1
python tools/pmc_traffic.py $O/pmc_m1 "k_expand_heavy<" k_expand_heavy m1 --out $O/traffic_m1.json || exit 1
timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print('c3', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['kernel'], round(d['roofline']['frac'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:6]})"
cat $O/traffic_m1.json
echo ALL_OK
