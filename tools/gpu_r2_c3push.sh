# Round 2: C3 — push for the level-2 frontier (PULL_DIV 1.2: level 2 push, level 3 pull) and all push (1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/c3push
mkdir -p $O
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:3]})"
}
run div20 OMX_BFS_PULL_DIV=20
run div1.2 OMX_BFS_PULL_DIV=1.2
run div1 OMX_BFS_PULL_DIV=1
echo ALL_OK
