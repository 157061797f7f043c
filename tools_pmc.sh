#!/bin/bash
# PMC passes for the fused match kernel (one rocprofv3 run per counter group; never combined
# with tracing).  Usage (on the GPU box): bash tools_pmc.sh <outdir>
set -u
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --cache /tmp/wlB"
timeout -k 10 300 python -u bench.py $ARGS > "$OUT/prime.json" 2> "$OUT/prime.err" || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- python -u bench.py $ARGS > "$OUT/p$i.log" 2>&1
  echo "pass $i ($grp) rc=$?"
done
