# march register budget A/B (alternate builds via PT_AMD_LIB): default (5 waves), 4 waves, 6 waves
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3k
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 24 > $OUT/bench_mw5.json 2> $OUT/bench_mw5.err
PT_AMD_LIB=$GRAFT_REPO_ROOT/rs-pathtracing_amd/variants/lib_mw4.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 24 > $OUT/bench_mw4.json 2> $OUT/bench_mw4.err
PT_AMD_LIB=$GRAFT_REPO_ROOT/rs-pathtracing_amd/variants/lib_mw6.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 24 > $OUT/bench_mw6.json 2> $OUT/bench_mw6.err
