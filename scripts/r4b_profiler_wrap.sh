set -e
export PROF_TIMEOUT=400
SQ_FRAMES=1 SQ_SAMPLES=8493465600 WORKLOAD="cornell_box.json 3840x2160 1024spp depth 8" PT_SEGV_LOG=$GRAFT_REPO_ROOT/gpurun_out/r4b/segv_c3s4.log bash scripts/gpu.sh sq r4b/sq_c3_slots4 --config c3 --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-roofline-leg --slots 4
echo c3s4 done > gpurun_out/r4b/progress.txt
SQ_FRAMES=2 bash scripts/gpu.sh sq r4b/sq_c2_slots1 --steps 2 --warmup 0 --no-cpu-baseline --no-parity --no-roofline-leg --slots 1
echo c2s1 done >> gpurun_out/r4b/progress.txt
SQ_FRAMES=12 PT_SEGV_LOG=$GRAFT_REPO_ROOT/gpurun_out/r4b/segv_c2_12.log bash scripts/gpu.sh sq r4b/sq_c2_12frames --steps 12 --warmup 0 --no-cpu-baseline --no-parity --no-roofline-leg --slots 1
echo c2x12 done >> gpurun_out/r4b/progress.txt
