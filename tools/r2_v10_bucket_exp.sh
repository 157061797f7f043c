# Round 2: retained walk with 128-B edge buckets + early word loads, search variants (0 fenced binary, 1 16-ary S-tree): parity of both,
# config R bench of both, and the walk's per-phase cycle split (RETAIN_PROF build).
set -o pipefail
O=gpurun_out/r2_v10
mkdir -p $O
for sv in 0 1; do
  EMQX_RETAIN_SEARCH=$sv timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_retain.py > $O/pytest_s$sv.log 2>&1
  rc=$?; echo "pytest search=$sv rc=$rc"; tail -1 $O/pytest_s$sv.log; [ $rc -eq 0 ] || exit $rc
done
for sv in 0 1; do
  EMQX_RETAIN_SEARCH=$sv timeout -k 10 300 python -u bench.py --workload R --steps 20 --warmup 3 --no-cpu-baseline > $O/benchR_s$sv.json 2> $O/benchR_s$sv.err
  rc=$?; echo "bench search=$sv rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/benchR_s$sv.err; exit $rc; }
  python -c "import json,sys; d=json.loads(open('$O/benchR_s$sv.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('ms_per_step','call_ms_median','walk_ms_median','walk_spill_rounds')})"
  EMQX_LIB=$PWD/emqx_amd/_build_prof/libemqxmatch.so EMQX_RETAIN_PROF=1 EMQX_RETAIN_SEARCH=$sv timeout -k 10 300 python -u bench.py --workload R --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_s$sv.json 2> $O/prof_s$sv.err
  rc=$?; echo "prof search=$sv rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_s$sv.err; exit $rc; }
  grep RETAIN_PROF $O/prof_s$sv.err | tail -3
done
