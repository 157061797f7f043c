#!/bin/bash
# Quick check of the tree on a GPU box: GPU tests, smoke, config-B bench line (with parity).
# Usage: bash tools/r2_check.sh <tag> [pytest-args...]
set -u -o pipefail
TAG=${1:-check}; shift || true
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/benchB.json 2> $O/benchB.err || { echo bench failed; tail -20 $O/benchB.err; exit 1; }
cat $O/benchB.json
