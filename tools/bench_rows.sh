#!/bin/bash
# The other bench lines (configs A, E and rows f2/f4: U, R) with default arguments.
set -e
TAG=${1:-rows}
O=gpurun_out/$TAG; mkdir -p $O
for w in A E U R; do
  echo "== $w"; date
  timeout -k 10 600 python -u bench.py --workload $w > $O/bench$w.json 2> $O/bench$w.err || { tail -20 $O/bench$w.err; exit 1; }
  cut -c1-400 $O/bench$w.json
done
