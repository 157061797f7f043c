# Config C's 100M-filter table on one GPU (C1): bench line, then FETCH_SIZE / WRITE_SIZE /
# TCC hit-miss passes of the fast kernel (C1 gets PMC traffic).  The workload
# is cached in /tmp/wlC by the first run; each run rebuilds the 23 GB table (~3 min).
# Usage: bash tools/r2_c1_pmc.sh <tag> <part: bench (bench + FETCH) | rest (WRITE + TCC)>
set -o pipefail
O=gpurun_out/${1:-r2_c1}
PART=${2:-bench}
mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
ARGS="--n-filters 100000000 --vocab-scale 4 --no-cpu-baseline --no-host-api --cache /tmp/wlC --streams 1"
if [ "$PART" = bench ]; then
  timeout -k 10 700 python -u bench.py $ARGS --steps 10 > $O/benchC1.json 2> $O/benchC1.err
  rc=$?; echo "bench rc=$rc"; tail -3 $O/benchC1.err; [ $rc -eq 0 ] || exit $rc
  GROUPS_="FETCH_SIZE"
else
  GROUPS_="WRITE_SIZE TCC_HIT_sum%TCC_MISS_sum"
fi
i=0
for grp in $GROUPS_; do
  i=$((i+1))
  g=${grp//%/ }
  cd /tmp
  timeout -s KILL 560 rocprofv3 --pmc $g --kernel-include-regex match_fast_kernel --output-format csv -d $ROOT/$O/pmc_${PART}_$i -o pmc -- python3 $ROOT/bench.py $ARGS --steps 3 --warmup 1 > $ROOT/$O/pmc_${PART}_$i.log 2>&1
  rc=$?; cd $ROOT; echo "pmc $g rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc_${PART}_$i.log; exit $rc; }
done
