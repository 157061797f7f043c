# Final round-1 check of the committed tree: GPU tests, smoke, config B and R bench lines.
set -o pipefail
O=gpurun_out/r1_v10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --workload R > $O/benchR.json 2> $O/benchR.err || { tail -20 $O/benchR.err; exit 1; }
timeout -k 10 600 python -u bench.py > $O/benchB.json 2> $O/benchB.err || { tail -20 $O/benchB.err; exit 1; }
python -c "import json; [print(n, json.load(open('$O/bench'+n+'.json'))['value']) for n in 'RB']"
