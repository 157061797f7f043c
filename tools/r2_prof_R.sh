# Kernel trace of config R (retained lookup): rocprofv3 --kernel-trace --stats into $1.
set -o pipefail
O=${1:-gpurun_out/r2_profR}
SV=${2:-1}
mkdir -p $O
ROOT=$(pwd)
cd /tmp
EMQX_RETAIN_SEARCH=$SV timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o prof -- python3 $ROOT/bench.py --workload R --no-cpu-baseline --steps 10 --warmup 2 > $ROOT/$O/prof.log 2>&1
rc=$?; cd $ROOT; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
python3 - "$O" <<'PY'
import csv, glob, sys
for p in glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
