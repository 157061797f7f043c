set -u
OUT=gpurun_out/${1:-r4_v12}
mkdir -p $OUT
bash tools/r4_v7.sh $1 || exit 1
timeout -k 10 300 python -u tools/single_publisher.py --strategy round_robin > $OUT/single_pub_rr.json 2> $OUT/single_pub_rr.err || { tail $OUT/single_pub_rr.err; exit 1; }
timeout -k 10 300 python -u tools/single_publisher.py --strategy sticky > $OUT/single_pub_sticky.json 2> $OUT/single_pub_sticky.err || { tail $OUT/single_pub_sticky.err; exit 1; }
cat $OUT/single_pub_*.json
timeout -k 10 500 python -u bench.py --workload T > $OUT/bench_T.json 2> $OUT/bench_T.err || { tail -20 $OUT/bench_T.err; exit 1; }
tail -c 3000 $OUT/bench_T.json
