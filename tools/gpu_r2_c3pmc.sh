# Round 2: C3 pull — varlen parity, the default C3 line, then its counters (FETCH/WRITE traffic, SQ
# issue and wait, L2 requests and hits) and a kernel-trace summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/c3final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAIL; grep -m2 -A40 "^____" $O/tests.log | head -60; exit 1; }
timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --cpu-seconds 10 > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3', round(d['value'],1), round(d['ms_per_step'],3), d['roofline'], {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]}, d['cpu_baseline']['value'])"
bash tools/pmc.sh k_bfs_pull $O --query c3 --steps 2 --warmup 1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_bfs_pull -d $O/p5 -o pmc --output-format csv \
  -- python3 bench.py --no-cpu-baseline --query c3 --steps 2 --warmup 1 > $O/p5.log 2>&1 || { echo "pass 5 failed"; tail -5 $O/p5.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv \
  -- python3 bench.py --no-cpu-baseline --query c3 --steps 5 --warmup 1 > $O/kt.log 2>&1 || { echo "kt failed"; exit 1; }
echo ALL_OK
