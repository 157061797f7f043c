# Config R with first-come tile assignment: tile size and walk waves (S-tree search).
O=gpurun_out/r2_tiles
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_retain.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
run() {
  i=$((i+1))
  env "$@" timeout -k 10 120 python -u bench.py --workload R --steps 10 --warmup 2 --no-cpu-baseline > $O/s$i.json 2> $O/s$i.err
  rc=$?
  python -c "import json,sys; d=json.loads(open('$O/s$i.json').read().strip().splitlines()[-1]); print('$*', {k: d.get(k) for k in ('call_ms_median','walk_ms_median','walk_spill_rounds','walk_spilled_items')})" 2>/dev/null || { echo "setting $* rc=$rc"; tail -3 $O/s$i.err; }
  [ $rc -eq 0 ] || exit $rc
}
run EMQX_RETAIN_TILE=8
run EMQX_RETAIN_TILE=4
run EMQX_RETAIN_TILE=6
run EMQX_RETAIN_TILE=12
run EMQX_RETAIN_TILE=8 EMQX_RETAIN_WALK_WAVES=6144
run EMQX_RETAIN_TILE=4 EMQX_RETAIN_WALK_WAVES=6144
run EMQX_RETAIN_TILE=6 EMQX_RETAIN_STEP_BUDGET=192
run EMQX_RETAIN_TILE=8 EMQX_RETAIN_STEP_BUDGET=192
# config D's per-level item histogram (is LDS staging of the upper levels worth it on D?)
timeout -k 10 300 python -u bench.py --workload D --diag --no-cpu-baseline --no-host-api --steps 3 --warmup 1 > $O/benchD_diag.json 2> $O/benchD_diag.err
rc=$?; echo "D diag rc=$rc"; python -c "import json; d=json.loads(open('$O/benchD_diag.json').read().strip().splitlines()[-1]); print(d.get('diag_per_topic')); print(d.get('diag_per_wave'))"
