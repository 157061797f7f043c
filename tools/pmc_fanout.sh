#!/bin/bash
# rocprofv3 --pmc passes over the fan-out kernels of bench.py --workload E (one counter group per
# run, never combined with tracing), then tools/pmc_fanout.py -> profiles/pmc_fanout_E.json.
# Also the FETCH_SIZE / WRITE_SIZE calibration of the fan-out's access widths (gather_bench cal).
# Usage (GPU box, repo root): bash tools/pmc_fanout.sh <outdir> [strategy]
set -u
OUT=${1:-gpurun_out/pmcE}; STRAT=${2:-hash_clientid}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
ARGS="--workload E --strategy $STRAT --steps 3 --warmup 1 --streams 1 --no-cpu-baseline"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-include-regex "fanout_" --output-format csv -d "$ROOT/$OUT/pmc$i" -o pmc -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/pmc$i.log" 2>&1
  rc=$?; cd "$ROOT"; echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/pmc$i.log"; exit $rc; }
done
python tools/pmc_fanout.py "$OUT" --strategy "$STRAT" > "$OUT/pmc_fanout.json"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "stream_|write_dword" --output-format csv -d "$ROOT/$OUT/cal1" -o cal -- "$ROOT/tools/_build/gather_bench" cal > "$ROOT/$OUT/cal1.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "stream_|write_dword" --output-format csv -d "$ROOT/$OUT/cal2" -o cal -- "$ROOT/tools/_build/gather_bench" cal > "$ROOT/$OUT/cal2.log" 2>&1
rc=$?; cd "$ROOT"; echo "calibration rc=$rc"
