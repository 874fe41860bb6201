# Round 2: C3 — push/pull switch point (OMX_BFS_PULL_DIV) and resident pull workgroups per CU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/c3dir
mkdir -p $O
run() {  # name, env...
  n=$1; shift
  env "$@" OMX_DEBUG_EXPAND=1 timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:3]})"
}
run div20 OMX_BFS_PULL_DIV=20
run div5 OMX_BFS_PULL_DIV=5
run div80 OMX_BFS_PULL_DIV=80
run div2 OMX_BFS_PULL_DIV=2
run per6 OMX_PULL_PER=6
run per8 OMX_PULL_PER=8
timeout -k 10 300 python -u tools/ridbag_bench.py --scale 22 > $O/ridbag.json 2> $O/ridbag.err || { tail $O/ridbag.err; exit 1; }
cat $O/ridbag.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ridbag -o rb --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ridbag_bench.py --scale 22 --reps 2 > $GRAFT_REPO_ROOT/$O/prof_ridbag.json 2> $GRAFT_REPO_ROOT/$O/prof_ridbag.err ) || { echo PROF_FAIL; tail $O/prof_ridbag.err; exit 1; }
echo ALL_OK
