#!/bin/bash
# SQ / TA / TCP counter passes for the fused match kernel, per fast-kernel variant (one
# rocprofv3 run per counter group, never combined with tracing).
# Usage (GPU box, repo root): bash tools/pmc_sq.sh <outdir> <variant> [<variant> ...]
set -u
OUT=${1:-gpurun_out/sq}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
[ -s "$OUT/counters.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-host-api --streams 1 --cache /tmp/wlB"
timeout -k 10 300 python -u bench.py $ARGS > "$OUT/prime.json" 2> "$OUT/prime.err" || { echo prime failed; exit 1; }
for v in "$@"; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" \
             "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
             "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    cd /tmp
    EMQX_FAST_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex match_fast_kernel --output-format csv -d "$ROOT/$OUT/v$v/p$i" -o pmc -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/v$v.p$i.log" 2>&1
    rc=$?; cd "$ROOT"; echo "variant $v pass $i rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/v$v.p$i.log"; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc; }
  done
  python tools/pmc_summary.py --dir "$OUT/v$v" --kernel match_fast_kernel > "$OUT/v$v.summary.json"
done
