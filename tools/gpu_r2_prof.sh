# Round 2: kernel-trace profiles of M1, C2, C1 (rocprofv3 --stats) and host phase traces.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/prof8
mkdir -p $O
for q in m1 c2 c1; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/$q -o $q --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --query $q --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/$q.json 2> $GRAFT_REPO_ROOT/$O/$q.err ) || { echo PROF_FAIL $q; tail $O/$q.err; exit 1; }
done
for q in m1 c2; do
  OMX_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --query $q --steps 3 --warmup 1 --no-cpu-baseline > $O/${q}_host.json 2> $O/${q}_host.err || exit 1
done
find $O -name "*kernel_stats.csv" | head
echo ALL_OK
