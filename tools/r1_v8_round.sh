set -o pipefail
bash tools/gpu_round.sh r1_v8 || exit 1
OUT=gpurun_out/r1_v8
timeout -k 10 400 python -u bench.py --workload R > $OUT/benchR.json 2> $OUT/benchR.err || { tail -20 $OUT/benchR.err; exit 1; }
cat $OUT/benchR.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/profR -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload R --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/profR.json 2> $GRAFT_REPO_ROOT/$OUT/profR.err || { tail -20 $GRAFT_REPO_ROOT/$OUT/profR.err; exit 1; }
echo done
