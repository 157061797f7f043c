# Round-1 closing check of the committed tree: all GPU tests, smoke, R kernel stats (rocprofv3).
set -o pipefail
O=gpurun_out/r1_v12c
mkdir -p $O
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/profR -o run -- python3 $ROOT/bench.py --workload R --no-cpu-baseline > $ROOT/$O/profR.json 2> $ROOT/$O/profR.err || { tail -20 $ROOT/$O/profR.err; exit 1; }
head -6 $ROOT/$O/profR/run_kernel_stats.csv | cut -c1-150
