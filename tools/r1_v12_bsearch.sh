# Paired lower bounds in the retained walk (round 1, v12): GPU retain tests, then the R bench.
set -o pipefail
O=gpurun_out/r1_v12
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_retain.py -x -v --timeout 120 --timeout-method thread > $O/pytest_retain.log 2>&1 || { tail -30 $O/pytest_retain.log; exit 1; }
tail -1 $O/pytest_retain.log
timeout -k 10 400 python -u bench.py --workload R > $O/benchR.json 2> $O/benchR.err || { tail -20 $O/benchR.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['walk_ms_median'], d['call_ms_median'], d['walk_spill_rounds'])" $O/benchR.json
