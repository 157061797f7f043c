mkdir -p gpurun_out/r4_v6
timeout -k 10 300 tools/_build/sort_bench > gpurun_out/r4_v6/sort_bench.jsonl 2>&1; echo "sort_bench rc=$?"
timeout -k 10 400 python -u -m pytest tests/test_gpu_share_parity.py tests/test_gpu_fanout_state.py tests/test_gpu_fanout.py -q --timeout 300 --timeout-method thread > gpurun_out/r4_v6/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4_v6/pytest.log
[ $rc -eq 0 ] || exit $rc
for st in hash_clientid round_robin sticky; do
  timeout -k 10 300 python -u bench.py --workload E --strategy $st --no-cpu-baseline > gpurun_out/r4_v6/bench_E_$st.json 2> gpurun_out/r4_v6/bench_E_$st.err || exit 1
done
for st in round_robin; do
  timeout -k 10 300 python -u bench.py --workload E --strategy $st --publishers 1 --no-cpu-baseline > gpurun_out/r4_v6/bench_E_${st}_pub1.json 2> gpurun_out/r4_v6/bench_E_${st}_pub1.err || exit 1
done
echo done
