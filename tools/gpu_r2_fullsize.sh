set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r1_fullsize.log 2>&1 || { echo FULLSIZE_FAIL; tail -30 gpurun_out/r1_fullsize.log; exit 1; }
tail -12 gpurun_out/r1_fullsize.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r1_bench_m1.json 2> gpurun_out/r1_bench_m1.err || { echo BENCH_FAIL; tail -20 gpurun_out/r1_bench_m1.err; exit 1; }
cat gpurun_out/r1_bench_m1.json
