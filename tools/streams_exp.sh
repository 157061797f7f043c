#!/bin/bash
# Pipelining experiment: per-step time vs number of HIP streams, configs D and B.
set -e
O=gpurun_out/streams; mkdir -p $O
for s in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload D --cache /tmp/wlD --no-cpu-baseline --streams $s --steps 12 > $O/d_s$s.json 2> $O/d_s$s.err
  python -c "import json;d=json.load(open('$O/d_s$s.json'));print('D streams $s', d['value'], d['ms_per_step'], d['call_ms_avg'])"
done
timeout -k 10 300 python -u bench.py --workload D --batch 250000 --no-cpu-baseline --streams 3 --steps 12 > $O/d250_s3.json 2> $O/d250.err
python -c "import json;d=json.load(open('$O/d250_s3.json'));print('D250k streams 3', d['value'], d['ms_per_step'], d['call_ms_avg'])"
timeout -k 10 300 python -u bench.py --workload D --batch 250000 --no-cpu-baseline --streams 1 --steps 12 > $O/d250_s1.json 2> $O/d250.err
python -c "import json;d=json.load(open('$O/d250_s1.json'));print('D250k streams 1', d['value'], d['ms_per_step'], d['call_ms_avg'])"
