#!/bin/bash
# Queue-walk occupancy A/B: the default build (4 waves per SIMD, 127 VGPRs) against builds
# compiled for 5 and 6 (96 / 80 VGPRs, with spills).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q23}
mkdir -p $OUT
for rep in 1 2; do
for v in default occ5 occ6; do
  if [ $v = default ]; then L=$(pwd)/emqx_amd/_build/libemqxmatch.so; else L=$(pwd)/emqx_amd/_build_$v/libemqxmatch.so; fi
  EMQX_LIB=$L timeout -k 10 200 python -u tools/retain_sweep.py --calls=20 'balance=1' > $OUT/$v.$rep.jsonl 2> $OUT/$v.$rep.err || { tail -20 $OUT/$v.$rep.err; exit 1; }
  echo "$v $rep $(cat $OUT/$v.$rep.jsonl)"
done
done
