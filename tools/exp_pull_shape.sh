# Experiment: C3 bench with pull-tile shape variants built into orientdb_amd/_exp/<bB_iIPT>/ and OMX_PULL_PER caps.
set -o pipefail
mkdir -p gpurun_out/exp
run() {  # name per
  OMX_PULL_PER=$2 timeout -k 10 150 python -u bench.py --query c3 --no-cpu-baseline > gpurun_out/exp/c3_$1_p$2.log 2>&1 || { tail -5 gpurun_out/exp/c3_$1_p$2.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/exp/c3_$1_p$2.log').read().strip().splitlines()[-1]); print('$1 per=$2', round(d['value']), round(d['ms_per_step'],3), d['kernels']['k_bfs_pull']['ms_per_step'])"
}
run base 7
for n in b256_i2 b128_i4; do
  cp orientdb_amd/_exp/$n/libomx.so orientdb_amd/_lib/libomx.so
  for p in 7 10 14 20; do run $n $p; done
done
