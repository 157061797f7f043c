#!/bin/bash
# Walk order experiment: GPU parity of the reordered walk, then D and B with the order off / on.
set -u -o pipefail
O=gpurun_out/r2_v22
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_order.py > $O/pytest_order.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_order.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-host-api"
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py $B "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -20 $O/$tag.err; exit 1; }
  python - $O/$tag.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["call_ms_avg"], d["roofline"]["kernel_ms_avg"], d["config"].get("walk_order"))
PY
}
run D_off --workload D --cache /tmp/wlD --walk-order off --steps 10
run D_on --workload D --cache /tmp/wlD --walk-order on --steps 10
run D_on_lb2 --workload D --cache /tmp/wlD --walk-order on --walk-level-bits 2 --steps 10
run D_on_nodeal --workload D --cache /tmp/wlD --walk-order on --walk-deal 0 --steps 10
run B_off --cache /tmp/wlB --walk-order off
run B_on --cache /tmp/wlB --walk-order on
run B_on_s16 --cache /tmp/wlB --walk-order on --walk-sort-bits 16
run B_on_s24 --cache /tmp/wlB --walk-order on --walk-sort-bits 24 --walk-level-bits 6
