# Output-stage ablations of config R (RETAIN_PROF build; results are wrong by design, timing
# only): kernel trace per ablation mask (1 no small rows, 2 no big records, 4 no atomics).
O=gpurun_out/r2_ablate
mkdir -p $O
ROOT=$(pwd)
for m in 0 1 2 4 7; do
  cd /tmp
  EMQX_LIB=$ROOT/emqx_amd/_build_prof/libemqxmatch.so EMQX_RETAIN_PROF=1 EMQX_RETAIN_ABLATE=$m EMQX_RETAIN_SEARCH=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/m$m -o prof -- python3 $ROOT/bench.py --workload R --no-cpu-baseline --steps 3 --warmup 1 > $ROOT/$O/m$m.log 2>&1
  rc=$?; cd $ROOT; echo "mask $m rc=$rc"
  python3 - "$O/m$m" <<'PY'
import csv, glob, sys
for p in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "out_kernel" in r["Name"] or "walk_kernel" in r["Name"]:
            print("  ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
done
