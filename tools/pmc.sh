#!/bin/bash
# PMC passes for one kernel of a bench run (one counter group per rocprofv3 run, as the MI355X guide
# prescribes: FETCH_SIZE and WRITE_SIZE in separate passes).
# usage: tools/pmc.sh <kernel-regex> <outdir> [bench args...]
set -o pipefail
K=$1; OUT=$2; shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $pmc --kernel-include-regex "$K" -d "$OUT/p$i" -o pmc --output-format csv \
    -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo pmc done
