#!/bin/bash
# 28-waves/CU variants (512 word ids, <= 72 VGPRs) against the default on config B, plus the
# variant parity tests.
set -e
O=gpurun_out/occ; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --cache /tmp/wlB --ab 7,11,12 --steps 30 --no-cpu-baseline > $O/ab.json 2> $O/ab.err
cat $O/ab.json
