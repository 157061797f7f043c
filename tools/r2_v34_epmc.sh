#!/bin/bash
# Config E fan-out kernels: where fanout_write waits (SQ), L2 behaviour and bytes (PMC passes).
set -u -o pipefail
O=gpurun_out/${1:-r2_v34}
mkdir -p $O
ROOT=$(pwd)
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex fanout_ --output-format csv -d $ROOT/$O/pmc$i -o pmc -- python3 $ROOT/bench.py --workload E --no-cpu-baseline --steps 3 --warmup 1 > $ROOT/$O/pmc$i.log 2>&1
  rc=$?; cd $ROOT; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc$i.log; exit $rc; }
done
python - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(O + "/pmc*/**/*counter_collection.csv", recursive=True):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        acc[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, d), cs in acc.items():
        for c, v in cs.items():
            per[k][c].append(v)
for k, cs in per.items():
    print(k, {c: f"{sorted(v)[len(v)//2]:.4g}" for c, v in cs.items()})
PY
