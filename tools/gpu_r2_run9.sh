# Round 2: TRAVERSE / SELECT expand() parity, factorized parity (wave-aggregated grouping), then M1 / C2 / C1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_traverse.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/trav.log 2>&1
rc=$?; tail -3 $O/trav.log
[ $rc -eq 0 ] || { echo TRAV_FAIL; grep -m2 -A40 "^____" $O/trav.log | head -60; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -3 $O/parity.log
[ $rc -eq 0 ] || { echo PARITY_FAIL; grep -m2 -A30 "^____" $O/parity.log | head -50; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/m1.json 2> $O/m1.err || { tail $O/m1.err; exit 1; }
timeout -k 10 300 python -u bench.py --query c2 --steps 20 --warmup 3 > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
timeout -k 10 300 python -u bench.py --query c1 --steps 20 --warmup 3 > $O/c1.json 2> $O/c1.err || { tail $O/c1.err; exit 1; }
for f in m1 c2 c1; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['kernel'], round(d['roofline']['frac'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:6]})"; done
echo ALL_OK
