# Round 2: round-end rehearsal — the whole GPU suite in one process, smoke(), the default bench line, P1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/full
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', round(d['value'],1), round(d['ms_per_step'],3), d['roofline'], d['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --query p1 --steps 10 --warmup 2 --cpu-seconds 8 > $O/p1.json 2> $O/p1.err || { tail $O/p1.err; exit 1; }
python -c "import json;d=json.load(open('$O/p1.json'));print('p1', round(d['value'],3), round(d['ms_per_step'],3), d['config']['rows_per_step'], {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]}, d['cpu_baseline'])"
echo ALL_OK
