#!/bin/bash
# Config D / deep-path experiment: variant and deep tests, then interleaved A/B of fast-kernel
# variants on config D (100k and 1M batches) and config B.
set -e
export TMPDIR=/tmp
O=gpurun_out/dexp; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload D --batch 100000 --ab 0,9,10,3 --no-cpu-baseline > $O/d100k.json 2> $O/d100k.err
cat $O/d100k.json
timeout -k 10 400 python -u bench.py --workload D --batch 1000000 --ab 0,9,10,3 --ab-rounds 2 --steps 4 --no-cpu-baseline > $O/d1m.json 2> $O/d1m.err
cat $O/d1m.json
timeout -k 10 400 python -u bench.py --cache /tmp/wlB --ab 7,9,10 --no-cpu-baseline > $O/b.json 2> $O/b.err
cat $O/b.json
