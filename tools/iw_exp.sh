#!/bin/bash
# A/B of the intern round width (IW words per lane): bench B with the in-tree build (IW=2),
# then rebuilt on the box with IW=1.
set -e
O=gpurun_out/iw; mkdir -p $O
timeout -k 10 300 python -u bench.py --cache /tmp/wlB --no-cpu-baseline --diag > $O/iw2.json 2> $O/iw2.err
python -c "import json;d=json.load(open('$O/iw2.json'));print('IW2', d['value'], d['roofline']['kernel_ms_avg'], d['call_ms_avg'], json.dumps(d['diag_per_wave']))"
sed -i 's/  constexpr uint32_t IW = 2;  /  constexpr uint32_t IW = 1;  /' emqx_amd/csrc/match_kernels.hip
make -C emqx_amd/csrc -j16 > $O/make.log 2>&1
timeout -k 10 300 python -u bench.py --cache /tmp/wlB --no-cpu-baseline --diag > $O/iw1.json 2> $O/iw1.err
python -c "import json;d=json.load(open('$O/iw1.json'));print('IW1', d['value'], d['roofline']['kernel_ms_avg'], d['call_ms_avg'], json.dumps(d['diag_per_wave']))"
