#!/bin/bash
# tests/test_gpu_c100m.py: config C's 100M table, replicated and sharded, ID-for-ID on 20K topics.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_c100m}
mkdir -p $OUT
EMQX_GPU_C100M=1 timeout -k 10 1150 python -u -m pytest -x -v --timeout 1100 --timeout-method thread \
  tests/test_gpu_c100m.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; cat gpurun_out/c100m_progress.log; exit 1; }
tail -3 $OUT/pytest.log
cp gpurun_out/c100m_progress.log $OUT/ 2>/dev/null; cat $OUT/c100m_progress.log | tail -8
