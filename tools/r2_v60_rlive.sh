# Round 2 retained lookup with live masks kept between the output passes: GPU tests, R bench, kernel
# trace, FETCH/WRITE PMC passes (-> pmc_retain.json).
set -o pipefail
O=gpurun_out/${1:-r2_v60}
mkdir -p $O
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_retain.py > $O/pytest_retain.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_retain.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload R --steps 20 --warmup 3 > $O/benchR.json 2> $O/benchR.err
rc=$?; echo "bench R rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/benchR.err; exit $rc; }
bash tools/r2_prof_R.sh $O/trace 1 || exit 1
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex retain_ --output-format csv -d $ROOT/$O/pmc$i -o pmc -- python3 $ROOT/bench.py --workload R --no-cpu-baseline --steps 5 --warmup 1 > $ROOT/$O/pmc$i.log 2>&1
  rc=$?; cd $ROOT; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/pmc$i.log; exit $rc; }
done
python tools/pmc_retain.py --dir $O --filters 100000 --retained 864333 --out $O/pmc_retain.json
