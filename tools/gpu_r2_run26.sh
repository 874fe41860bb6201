# Round 2: TRAVERSE / shortestPath on the reference's known-answer graph; P1 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r26
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_traverse.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
[ $rc -eq 0 ] || { echo TEST_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -70; exit 1; }
timeout -k 10 400 python -u bench.py --query p1 --steps 10 --warmup 2 --cpu-seconds 8 > $O/p1.json 2> $O/p1.err || { tail $O/p1.err; exit 1; }
python -c "import json;d=json.load(open('$O/p1.json'));print('p1', round(d['value'],3), round(d['ms_per_step'],3), d['config']['query'], d['config']['rows_per_step'], d['config']['edges_per_step'], {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]}, d['cpu_baseline'])"
echo ALL_OK
