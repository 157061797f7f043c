set -u
OUT=gpurun_out/${1:-r4_v7}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_share_parity.py tests/test_gpu_fanout_state.py tests/test_gpu_fanout.py -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/pytest.log | head -20; exit $rc; }
for st in hash_clientid round_robin sticky; do
  timeout -k 10 300 python -u bench.py --workload E --strategy $st --no-cpu-baseline > $OUT/bench_E_$st.json 2> $OUT/bench_E_$st.err || exit 1
done
for p in 1 1000; do
  timeout -k 10 300 python -u bench.py --workload E --strategy round_robin --publishers $p --no-cpu-baseline > $OUT/bench_E_rr_pub$p.json 2> $OUT/bench_E_rr_pub$p.err || exit 1
done
for f in $OUT/bench_E_*.json; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', round(d['value']/1e9,3), 'G topics/s', d['ms_per_step'], 'ms/step fo', d['fanout_call_ms'])"; done
