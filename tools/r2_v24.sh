#!/bin/bash
# Rehearsal of bench.py's N-rank path (2 ranks sharing the box's GPU over gloo), then D with
# the host enqueue timing, then rocprof kernel stats of D.
set -u -o pipefail
O=gpurun_out/r2_v24
mkdir -p $O
export EMQX_BENCH_REHEARSE=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --n-filters 1000000 > $O/rehearse2.json 2> $O/rehearse2.err || { echo rehearsal failed; tail -30 $O/rehearse2.err; exit 1; }
tail -1 $O/rehearse2.json | cut -c1-500
unset EMQX_BENCH_REHEARSE
timeout -k 10 600 python -u bench.py --workload D --cache /tmp/wlD --steps 10 --no-cpu-baseline --no-host-api > $O/benchD.json 2> $O/benchD.err || { echo D failed; tail -20 $O/benchD.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchD.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['host_enqueue_ms_per_step'], d['step_completion_gap_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/profD -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload D --cache /tmp/wlD --steps 5 --warmup 2 --no-cpu-baseline --no-host-api > $GRAFT_REPO_ROOT/$O/profD.json 2> $GRAFT_REPO_ROOT/$O/profD.err || { echo rocprof failed; tail -20 $GRAFT_REPO_ROOT/$O/profD.err; exit 1; }
cd $GRAFT_REPO_ROOT
find $O/profD -name "*kernel_stats.csv" -exec head -20 {} \;
