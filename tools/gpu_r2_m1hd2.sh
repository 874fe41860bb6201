# Round 2: M1 / C2 — the sliced (filtered) heavy cut with the unfiltered emission cut held at 1024.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/m1hd2
mkdir -p $O
run() {  # name, query, env...
  n=$1; q=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --query $q --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]})"
}
run m1_default m1
for h in 512 1024 4096 8192; do run m1_s$h m1 OMX_HEAVY_DEG=$h OMX_HEAVY_DEG_UNFILTERED=1024; done
for h in 256 512 1024; do run c2_s$h c2 OMX_HEAVY_DEG=$h OMX_HEAVY_DEG_UNFILTERED=1024; done
run c2_default c2
echo ALL_OK
