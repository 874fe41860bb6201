# Round 2: C3 pull — hub-array size sweep (OMX_PULL_HUBS) and resident workgroups per CU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/c3hubs
mkdir -p $O
for h in 262144 1048576 4194304 16777216; do
  for per in 7; do
    OMX_PULL_HUBS=$h OMX_PULL_PER=$per timeout -k 10 300 python -u bench.py --query c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/h${h}_p$per.json 2> $O/h${h}_p$per.err || { tail $O/h${h}_p$per.err; exit 1; }
    python -c "import json;d=json.load(open('$O/h${h}_p$per.json'));print('hubs $h per $per', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in list(d['kernels'].items())[:5]})"
  done
done
echo ALL_OK
