#!/bin/bash
# Config D (walk order on, the default) fast-kernel PMC passes -> pmc_summary.json, plus the
# FETCH_SIZE calibration, for tools/update_traffic.py --workload D.
set -u -o pipefail
O=gpurun_out/${1:-r2_dpmc}
mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
ARGS="--workload D --cache /tmp/wlD --no-cpu-baseline --no-host-api --streams 1"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o run -- python3 $ROOT/bench.py $ARGS --steps 5 --warmup 2 > $ROOT/$O/prof_bench.json 2> $ROOT/$O/prof_bench.err || { echo rocprof failed; tail -5 $ROOT/$O/prof_bench.err; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex match_fast_kernel --output-format csv -d $ROOT/$O/pmc$i -o pmc -- python3 $ROOT/bench.py $ARGS --steps 3 --warmup 1 > $ROOT/$O/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $ROOT/$O/pmc$i.log; exit $rc; }
done
cd $ROOT
python tools/pmc_summary.py --dir $O --kernel match_fast_kernel > $O/pmc_summary.json
if [ -x tools/_build/gather_bench ]; then
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_MISS_sum --kernel-include-regex indep_kernel --output-format csv -d $ROOT/$O/cal -o cal -- $ROOT/tools/_build/gather_bench > $ROOT/$O/cal.log 2>&1
  rc=$?; cd $ROOT; echo "calibration rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
cat $O/pmc_summary.json
