# Config R: step budget, spill dealing, spill waves and tile sweep (S-tree search).
O=gpurun_out/r2_budget
mkdir -p $O
i=0
run() {
  i=$((i+1))
  env EMQX_RETAIN_SEARCH=1 "$@" timeout -k 10 120 python -u bench.py --workload R --steps 10 --warmup 2 --no-cpu-baseline > $O/s$i.json 2> $O/s$i.err
  rc=$?
  python -c "import json,sys; d=json.loads(open('$O/s$i.json').read().strip().splitlines()[-1]); print('$*', {k: d.get(k) for k in ('call_ms_median','walk_ms_median','walk_spill_rounds','walk_spilled_items')})" 2>/dev/null || { echo "setting $* rc=$rc"; tail -3 $O/s$i.err; }
  [ $rc -eq 0 ] || exit $rc
}
run EMQX_RETAIN_STEP_BUDGET=128
run EMQX_RETAIN_STEP_BUDGET=64
run EMQX_RETAIN_STEP_BUDGET=96
run EMQX_RETAIN_STEP_BUDGET=192
run EMQX_RETAIN_STEP_BUDGET=256
run EMQX_RETAIN_SPILL_WAVES=2048
run EMQX_RETAIN_SPILL_WAVES=3072
run EMQX_RETAIN_SPILL_PER_WAVE=2
run EMQX_RETAIN_SPILL_PER_WAVE=8
run EMQX_RETAIN_SPILL_PER_WAVE=16
run EMQX_RETAIN_TILE=4
run EMQX_RETAIN_TILE=12
run EMQX_RETAIN_TILE=16
