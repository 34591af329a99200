# march 3/4-wave builds; bounce waves 2/4 with the 4-wave march (PT_WF_BOUNCE_WAVES picks a compiled variant)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3l
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/rs-pathtracing_amd/variants
PT_AMD_LIB=$L/lib_mw3.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 24 > $OUT/bench_mw3.json 2> $OUT/bench_mw3.err
PT_AMD_LIB=$L/lib_mw4.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 24 > $OUT/bench_mw4.json 2> $OUT/bench_mw4.err
PT_AMD_LIB=$L/lib_mw4.so PT_WF_BOUNCE_WAVES=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > $OUT/bench_mw4_bw2.json 2> $OUT/bench_mw4_bw2.err
PT_AMD_LIB=$L/lib_mw4.so PT_WF_BOUNCE_WAVES=4 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > $OUT/bench_mw4_bw4.json 2> $OUT/bench_mw4_bw4.err
PT_AMD_LIB=$L/lib_mw4.so PT_WF_MARCH_SLICE=128 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > $OUT/bench_mw4_s128.json 2> $OUT/bench_mw4_s128.err
