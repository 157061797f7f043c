# Config R: walk / spill wave counts, search variant and an occupancy-5 build of the walk
# kernels (emqx_amd/_build_occ5, -DRW_OCC=5): call and walk medians per setting.
O=gpurun_out/r2_waves
mkdir -p $O
i=0
run() {
  i=$((i+1))
  env "$@" timeout -k 10 120 python -u bench.py --workload R --steps 10 --warmup 2 --no-cpu-baseline > $O/s$i.json 2> $O/s$i.err
  rc=$?
  python -c "import json,sys; d=json.loads(open('$O/s$i.json').read().strip().splitlines()[-1]); print('$*', {k: d.get(k) for k in ('call_ms_median','walk_ms_median')})" 2>/dev/null || { echo "setting $* rc=$rc"; tail -3 $O/s$i.err; }
  [ $rc -eq 0 ] || exit $rc
}
OCC=EMQX_LIB=$PWD/emqx_amd/_build_occ5/libemqxmatch.so
run EMQX_RETAIN_SEARCH=1
run EMQX_RETAIN_SEARCH=1 EMQX_RETAIN_SPILL_WAVES=8192
run EMQX_RETAIN_SEARCH=1 EMQX_RETAIN_SPILL_WAVES=16384
run EMQX_RETAIN_SEARCH=1 EMQX_RETAIN_WALK_WAVES=4096
run EMQX_RETAIN_SEARCH=1 EMQX_RETAIN_WALK_WAVES=12800
run EMQX_RETAIN_SEARCH=0
run EMQX_RETAIN_SEARCH=0 EMQX_RETAIN_SPILL_WAVES=8192
run $OCC EMQX_RETAIN_SEARCH=1
run $OCC EMQX_RETAIN_SEARCH=1 EMQX_RETAIN_SPILL_WAVES=8192
run $OCC EMQX_RETAIN_SEARCH=1 EMQX_RETAIN_WALK_WAVES=5120 EMQX_RETAIN_SPILL_WAVES=5120
run $OCC EMQX_RETAIN_SEARCH=0
run $OCC EMQX_RETAIN_SEARCH=0 EMQX_RETAIN_SPILL_WAVES=8192
