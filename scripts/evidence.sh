#!/bin/bash
# Round evidence on one GPU box, every GPU step under its own time limit, the
# first failure ends the run (set -e).  Output: gpurun_out/<tag>/...
#
#   bash scripts/evidence.sh <tag> [pmc|bench|kt|all]
#
# pmc:   per config (c2, c3, c5) one SQ pass (f64 instruction counters ->
#        pmc_flops.json) and the FETCH_SIZE / WRITE_SIZE passes (-> pmc_traffic.json),
#        each over one one-stream frame of bench.py; the JSONs name the build
#        (source_id) so bench.py uses them only for that build.
# bench: bench.py lines for c1, c2 (default), c3, c5 with parity and CPU baseline.
# kt:    rocprofv3 --kernel-trace --stats of the default bench (+ one-stream leg).
set -e
tag=$1; what=${2:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
ONE="--steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-roofline-leg --slots 1"
declare -A SAMPLES=([c2]=530841600 [c3]=8493465600 [c5]=530841600)
declare -A WL=([c2]="cornell_box.json 1920x1080 256spp depth 8" [c3]="cornell_box.json 3840x2160 1024spp depth 8"
               [c5]="synthetic_100000 1920x1080 256spp depth 8")
if [ "$what" = pmc ] || [ "$what" = all ]; then
    for c in ${PMC_CONFIGS:-c2 c5 c3}; do
        # c3 (~4,000 dispatches per frame): counters on the render kernels only (unfiltered, rocprofv3 crashed)
        F=""; if [ $c = c3 ]; then F="wf_bounce|wf_march"; fi
        # c5 runs the FMA_SLAB bounce build: its FMAs beyond the expansions' 6.32 per TRANS are algorithmic
        R=""; if [ $c = c5 ]; then R=6.32; fi
        PMC_FMA_PER_TRANS="$R" PMC_FILTER="$F" WORKLOAD="${WL[$c]}" SQ_FRAMES=1 SQ_SAMPLES=${SAMPLES[$c]} PROF_TIMEOUT=300 \
            bash scripts/gpu.sh sq $tag/pmc_$c --config $c $ONE
        PMC_FILTER="$F" WORKLOAD="${WL[$c]}" PROF_TIMEOUT=300 bash scripts/gpu.sh pmc $tag/pmc_$c --config $c $ONE
        echo "pmc $c done" >> $OUT/progress.txt
    done
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
    echo "bench c2 done" >> $OUT/progress.txt
    timeout -k 10 300 python -u bench.py --config c1 --steps 20 --warmup 2 > $OUT/bench_c1.json 2> $OUT/bench_c1.err
    timeout -k 10 600 python -u bench.py --config c3 --steps 2 --warmup 1 > $OUT/bench_c3.json 2> $OUT/bench_c3.err
    echo "bench c3 done" >> $OUT/progress.txt
    timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
    echo "bench c5 done" >> $OUT/progress.txt
fi
if [ "$what" = kt ] || [ "$what" = all ]; then
    PROF_TIMEOUT=400 bash scripts/gpu.sh kt $tag/kt_default --no-cpu-baseline --no-parity
    echo "kt done" >> $OUT/progress.txt
fi
