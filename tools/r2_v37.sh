#!/bin/bash
# Walk-order key windows: order + parity GPU tests, then the D line (three streams, CPU baseline, parity).
set -u -o pipefail
O=gpurun_out/${1:-r2_v37}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_order.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py --workload D --cache /tmp/wlD --steps 10 > $O/benchD.json 2> $O/benchD.err || { echo D failed; tail -20 $O/benchD.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchD.json').read().strip().splitlines()[-1]); print('D', d['value'], d['ms_per_step'], d['call_ms_avg'], d['roofline']['kernel_ms_avg'], d['order_ms_avg'], d.get('parity'), d['cpu_baseline']['value'])"
