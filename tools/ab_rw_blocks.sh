set -u
OUT=gpurun_out/r5_rw1; mkdir -p $OUT
EMQX_LIB=$PWD/emqx_amd/_build_alt/libemqxmatch.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_retain.py > $OUT/pytest_alt.log 2>&1 || { tail -5 $OUT/pytest_alt.log; exit 1; }
tail -1 $OUT/pytest_alt.log
for r in 1 2 3 4; do for v in def alt; do
  if [ $v = alt ]; then L=$PWD/emqx_amd/_build_alt/libemqxmatch.so; else L=$PWD/emqx_amd/_build/libemqxmatch.so; fi
  EMQX_LIB=$L timeout -k 10 300 python bench.py --workload R --no-cpu-baseline > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail -5 $OUT/${v}_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['call_ms_median'], d.get('walk_ms_median'))" $OUT/${v}_$r.json "$v r=$r"
done; done
