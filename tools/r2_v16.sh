# Round 2: retained lookup, run-aggregated per-filter atomics: parity (both searches), R bench, kernel trace.
set -o pipefail
O=gpurun_out/r2_v16
mkdir -p $O
for sv in 0 1; do
  EMQX_RETAIN_SEARCH=$sv timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_retain.py > $O/pytest_s$sv.log 2>&1
  rc=$?; echo "pytest search=$sv rc=$rc"; tail -1 $O/pytest_s$sv.log; [ $rc -eq 0 ] || exit $rc
done
EMQX_RETAIN_SEARCH=1 timeout -k 10 300 python -u bench.py --workload R --steps 20 --warmup 3 --no-cpu-baseline > $O/benchR.json 2> $O/benchR.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/benchR.err; exit $rc; }
python -c "import json; d=json.loads(open('$O/benchR.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('ms_per_step','call_ms_median','walk_ms_median','walk_spill_rounds')})"
bash tools/r2_prof_R.sh $O/trace 1
