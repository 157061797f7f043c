#!/bin/bash
# PMC passes over the round-4 fan-out kernels (E, hash_clientid) -> profiles/pmc_fanout_E.json
# content (copied back from gpurun_out); S and T with the pooled commit patch building.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v20}
mkdir -p $OUT
bash tools/pmc_fanout.sh $OUT/pmcE hash_clientid > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
tail -3 $OUT/pmc.log
python3 -c "import json;d=json.load(open('$OUT/pmcE/pmc_fanout.json'));print('traffic per call', d['traffic_bytes_per_call'])"
timeout -k 10 300 python -u bench.py --workload S > $OUT/bench_S.json 2> $OUT/bench_S.err || { tail -20 $OUT/bench_S.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_S.json'));print('S',d['value'],d['ms_per_step'],d['host_ms_p50'],d['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --workload T > $OUT/bench_T.json 2> $OUT/bench_T.err || { tail -20 $OUT/bench_T.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_T.json'));print('T single', d['single_op']); [print(r['callers'], r['ops_per_s'], r['p99_us']) for r in d['storm']]; print(d['publish_alone'], d['publish_during_storm']['messages_per_s'])"
timeout -k 10 400 python -u bench.py --workload R > $OUT/bench_R.json 2> $OUT/bench_R.err || { tail -20 $OUT/bench_R.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_R.json'));print('R', d['value'], d['ms_per_step'])"
