# PMC passes (FETCH_SIZE, WRITE_SIZE, one run each) over config R's retain_* kernels, summed per
# call by tools/pmc_retain.py into profiles-ready JSON.
set -o pipefail
O=gpurun_out/r1_v10_pmcR
mkdir -p $O
ROOT=$(pwd)
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex retain_ --output-format csv -d $ROOT/$O/pmc$i -o pmc -- python3 $ROOT/bench.py --workload R --no-cpu-baseline --steps 5 --warmup 1 > $ROOT/$O/pmc$i.log 2>&1
  rc=$?; cd $ROOT; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/pmc$i.log; exit $rc; }
done
python tools/pmc_retain.py --dir $O --filters 100000 --retained 864333 --out $O/pmc_retain.json
