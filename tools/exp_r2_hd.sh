# RMAT-24 2-hop: heavy-row degree cut of the sliced kernels (P = 16 slices), one bench line per value,
# plus the binning debug line and a rocprofv3 kernel-stats pass of the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/hd
OMX_DEBUG_EXPAND=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/hd/debug.json 2> gpurun_out/hd/debug.err || exit 1
for hd in 256 512 1024 2048 4096; do
  OMX_HEAVY_DEG=$hd timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/hd/hd_$hd.json 2> gpurun_out/hd/hd_$hd.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hd/hd_$hd.json'));print($hd, round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in d['kernels'].items()})"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/hd/prof -o m1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/hd/prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/hd/prof -name "*kernel_stats*" | head -3
