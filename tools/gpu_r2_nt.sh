# Round 2: M1 with non-temporal dense-row stores (OMX_NT_STORES build in orientdb_amd/_lib_nt) vs default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/nt
mkdir -p $O
run() {  # name, query, env...
  n=$1; q=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --query $q --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:4]})"
}
run m1_plain m1
run m1_nt m1 OMX_LIB=$GRAFT_REPO_ROOT/orientdb_amd/_lib_nt/libomx.so
run m1_plain2 m1
run m1_nt2 m1 OMX_LIB=$GRAFT_REPO_ROOT/orientdb_amd/_lib_nt/libomx.so
run c1_plain c1
run c1_nt c1 OMX_LIB=$GRAFT_REPO_ROOT/orientdb_amd/_lib_nt/libomx.so
echo ALL_OK
