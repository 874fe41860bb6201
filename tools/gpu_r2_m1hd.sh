# Round 2: M1 / C2 — heavy-row cut of the unfiltered (emission) expansions.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/m1hd
mkdir -p $O
run() {  # name, query, env...
  n=$1; q=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --query $q --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]})"
}
for h in 1024 512 256 128; do run m1_h$h m1 OMX_HEAVY_DEG_UNFILTERED=$h; done
for h in 1024 256; do run c2_h$h c2 OMX_HEAVY_DEG_UNFILTERED=$h; done
echo ALL_OK
