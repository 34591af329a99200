set -e
mkdir -p gpurun_out/r1i
timeout -k 10 400 python -m pytest tests -q -x -m gpu > gpurun_out/r1i/pytest.log 2>&1
timeout -k 10 300 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1i/bench_wave64.log 2>&1
PT_ENGINE=mega timeout -k 10 300 python bench.py --spp 16 --steps 1 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/r1i/bench_mega16.log 2>&1
