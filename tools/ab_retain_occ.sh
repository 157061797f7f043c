#!/bin/bash
# Interleaved A/B of the retained walk's occupancy builds (QW_OCC 4 / 5 / 6) on config R.
set -u
O=gpurun_out/r6_qw; mkdir -p $O
for r in 1 2 3; do
  for q in 4 5 6; do
    L=emqx_amd/_build/libemqxmatch.so; [ $q != 4 ] && L=emqx_amd/_build_qw$q/libemqxmatch.so
    EMQX_LIB=$L timeout -k 10 300 python bench.py --workload R --no-cpu-baseline > $O/qw${q}_$r.json 2> $O/qw${q}_$r.err || { tail -20 $O/qw${q}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: d[k] for k in ('ms_per_step','call_ms_median') if k in d})" $O/qw${q}_$r.json "qw=$q r=$r"
  done
done
