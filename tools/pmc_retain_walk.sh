#!/bin/bash
# SQ / TA / TCP / TCC counter passes for the retained walk kernel (config R), one rocprofv3
# run per counter group, never combined with tracing.
# Usage (GPU box, repo root): bash tools/pmc_retain_walk.sh <outdir> [search variant]
set -u
OUT=${1:-gpurun_out/pmc_walk}
SV=${2:-1}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
ARGS="--workload R --steps 3 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" \
           "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  cd /tmp
  EMQX_RETAIN_SEARCH=$SV timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex retain_walk_kernel --output-format csv -d "$ROOT/$OUT/p$i" -o pmc -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.log" 2>&1
  rc=$?; cd "$ROOT"; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python tools/pmc_summary.py --dir "$OUT" --kernel retain_walk_kernel > "$OUT/summary.json"
cat "$OUT/summary.json"
