# Config R, first-come tiles: second sweep of tile size / walk waves (20 steps each).
O=gpurun_out/r2_tiles2
mkdir -p $O
i=0
run() {
  i=$((i+1))
  env "$@" timeout -k 10 120 python -u bench.py --workload R --steps 20 --warmup 3 --no-cpu-baseline > $O/s$i.json 2> $O/s$i.err
  rc=$?
  python -c "import json,sys; d=json.loads(open('$O/s$i.json').read().strip().splitlines()[-1]); print('$*', {k: d.get(k) for k in ('call_ms_median','walk_ms_median','walk_spill_rounds','walk_spilled_items')})" 2>/dev/null || { echo "setting $* rc=$rc"; tail -3 $O/s$i.err; }
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
run EMQX_RETAIN_TILE=8
run EMQX_RETAIN_TILE=10
run EMQX_RETAIN_TILE=12
run EMQX_RETAIN_TILE=14
run EMQX_RETAIN_TILE=16
run EMQX_RETAIN_TILE=8 EMQX_RETAIN_WALK_WAVES=6144
run EMQX_RETAIN_TILE=12 EMQX_RETAIN_WALK_WAVES=6144
done
