# Round-2 GPU check: the whole -m gpu suite (fail-fast), then the headline bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/suite.log 2>&1
rc=$?
tail -25 gpurun_out/suite.log
[ $rc -eq 0 ] || { echo SUITE_FAIL rc=$rc; exit 1; }
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_m1.json 2> gpurun_out/bench_m1.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_m1.err; exit 1; }
cat gpurun_out/bench_m1.json
