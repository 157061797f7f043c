# Phase cycles of the retained lookup's output kernels (RETAIN_PROF build), config R.
O=gpurun_out/r2_outprof
mkdir -p $O
EMQX_LIB=$PWD/emqx_amd/_build_prof/libemqxmatch.so EMQX_RETAIN_PROF=1 EMQX_RETAIN_SEARCH=1 timeout -k 10 300 python -u bench.py --workload R --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.json 2> $O/prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
grep RETAIN_ $O/prof.err | tail -6
