# Round 2: TRAVERSE fused (¬history ∧ WHILE) ordered filtered expansion: parity (traverse, parity, dist) + T1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r17
mkdir -p $O
for f in traverse dist parity; do
  timeout -k 10 400 python -u -m pytest tests/test_gpu_$f.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/$f.log 2>&1
  rc=$?; tail -1 $O/$f.log
  [ $rc -eq 0 ] || { echo FAIL $f; grep -m2 -A40 "^____" $O/$f.log | head -60; exit 1; }
done
for q in t1 s1; do
  timeout -k 10 400 python -u bench.py --query $q --steps 5 --warmup 2 --cpu-seconds 8 > $O/$q.json 2> $O/$q.err || { tail $O/$q.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$q.json'));print('$q', round(d['value'],1), round(d['ms_per_step'],3), d['config']['rows_per_step'], d['roofline']['kernel'], round(d['roofline']['frac'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:5]}, d['cpu_baseline']['value'], d['cpu_baseline']['sample'])"
done
echo ALL_OK
