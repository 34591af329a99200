#!/bin/bash
# Round evidence on one GPU box, every GPU step under its own time limit, the
# first failure ends the run (set -e).  Output: gpurun_out/<tag>/...
#
#   bash scripts/evidence.sh <tag> [pmc|bench|kt|all]
#
# pmc:   per config (c2, c3, c5) one SQ pass (f64 instruction counters ->
#        pmc_flops.json) and the FETCH_SIZE / WRITE_SIZE passes (-> pmc_traffic.json),
#        each over one frame of bench.py (one chunk stream; c3 at four: one stream
#        would queue ~8,300 dispatches on one HSA queue, profiles/r4/c3_profiler_abort.txt);
#        the JSONs name the build (source_id) so bench.py uses them only for that build,
#        for any frame size and spp of the same scene and depth (c4 uses c2/c3's).
# stall:  SQ wave-cycle split (active / memory wait / issue-stalled) of c2 and c5 one-stream frames.
# bench: bench.py lines for c1, c2 (default), c3, c4, c5 with parity and CPU baseline, c2 and c1 at depth 50,
#        the interactive workload (scripts/interactive_bench.py),
#        and c2 / c4 through 8 gloo ranks sharing the GPU (the multi-rank path).
# kt:    rocprofv3 --kernel-trace --stats of the default bench (+ one-stream leg).
# ranksim: scripts/rank_sim.py for c2 and c4 (per-rank shares, gather bounded by the link rate).
set -e
tag=$1; what=${2:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
ONE="--steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-roofline-leg --no-kernel-timing"
declare -A SAMPLES=([c2]=530841600 [c3]=8493465600 [c5]=530841600 [c2d50]=530841600)
declare -A WL=([c2]="cornell_box.json 1920x1080 256spp depth 8" [c3]="cornell_box.json 3840x2160 1024spp depth 8"
               [c5]="synthetic_100000 1920x1080 256spp depth 8" [c2d50]="cornell_box.json 1920x1080 256spp depth 50")
# bench arguments per config name (c2d50: the reference GUI's depth on the C2 frame)
declare -A CARGS=([c2]="--config c2" [c3]="--config c3" [c5]="--config c5" [c2d50]="--config c2 --depth 50")
if [ "$what" = pmc ] || [ "$what" = all ]; then
    for c in ${PMC_CONFIGS:-c2 c5 c3 c2d50}; do
        S=1; if [ $c = c3 ]; then S=4; fi
        # c5 runs the FMA_SLAB bounce build: its f64 FMAs beyond the expansions' 6.32 per TRANS are algorithmic
        R=""; if [ $c = c5 ]; then R=6.32; fi
        PMC_FMA_PER_TRANS="$R" WORKLOAD="${WL[$c]}" SQ_FRAMES=1 SQ_SAMPLES=${SAMPLES[$c]} PROF_TIMEOUT=300 \
            bash scripts/gpu.sh sq $tag/pmc_$c ${CARGS[$c]} $ONE --slots $S
        WORKLOAD="${WL[$c]}" PROF_TIMEOUT=300 bash scripts/gpu.sh pmc $tag/pmc_$c ${CARGS[$c]} $ONE --slots $S
        echo "pmc $c done" >> $OUT/progress.txt
    done
fi
if [ "$what" = stall ] || [ "$what" = all ]; then
    # wave-cycle split (active / waiting on memory / issue-stalled) of the one-stream frame
    for c in ${STALL_CONFIGS:-c2 c5}; do
        PROF_TIMEOUT=300 bash scripts/gpu.sh stall $tag/stall_$c ${CARGS[$c]} $ONE --slots 1
        echo "stall $c done" >> $OUT/progress.txt
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
    # the reference GUI's depth (informational: the configs are quoted at depth 8)
    timeout -k 10 600 python -u bench.py --depth 50 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c2_depth50.json \
        2> $OUT/bench_c2_depth50.err
    timeout -k 10 300 python -u bench.py --config c1 --depth 50 --steps 20 --warmup 2 --no-cpu-baseline \
        > $OUT/bench_c1_depth50.json 2> $OUT/bench_c1_depth50.err
    timeout -k 10 300 python -u scripts/interactive_bench.py --out $OUT/interactive.jsonl > $OUT/interactive.log 2>&1
    echo "bench depth 50 + interactive done" >> $OUT/progress.txt
fi
if [ "$what" = bench4 ] || [ "$what" = all ]; then
    timeout -k 10 900 python -u bench.py --config c4 --steps 1 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
    echo "bench c4 done" >> $OUT/progress.txt
    for c in c2 c4; do
        st=3; if [ $c = c4 ]; then st=1; fi
        timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
            --master-port 29517 bench.py --gpus 8 --dist-backend gloo --config $c --steps $st --warmup 1 \
            > $OUT/bench_${c}_gloo8.json 2> $OUT/bench_${c}_gloo8.err
        echo "bench $c gloo8 done" >> $OUT/progress.txt
    done
fi
if [ "$what" = ranksim ]; then
    timeout -k 10 600 python -u scripts/rank_sim.py --worlds 1,2,4,8 > $OUT/rank_sim_c2.txt 2>&1
    echo "ranksim c2 done" >> $OUT/progress.txt
    timeout -k 10 900 python -u scripts/rank_sim.py --worlds 1,8 --width 3840 --height 2160 --spp 4096 --reps 1 \
        > $OUT/rank_sim_c4.txt 2>&1
    echo "ranksim c4 done" >> $OUT/progress.txt
fi
if [ "$what" = kt ] || [ "$what" = all ]; then
    PROF_TIMEOUT=400 bash scripts/gpu.sh kt $tag/kt_default --no-cpu-baseline --no-parity --no-kernel-timing
    echo "kt done" >> $OUT/progress.txt
fi
