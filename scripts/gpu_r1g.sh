set -e
mkdir -p gpurun_out/r1g
for cfg in "1 65" "8 4" "16 8" "24 12" "32 16" "16 1" "32 8" "48 24" "16 16"; do
  set -- $cfg
  echo "trig=$1 keep=$2" >> gpurun_out/r1g/sweep.log
  PT_MARCH_TRIGGER=$1 PT_MARCH_KEEP=$2 timeout -k 10 120 python scripts/phase_profile.py 16 >> gpurun_out/r1g/sweep.log 2>&1
done
timeout -k 10 300 python -m pytest tests -q -x -m gpu > gpurun_out/r1g/pytest.log 2>&1
