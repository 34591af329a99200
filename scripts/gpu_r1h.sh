set -e
mkdir -p gpurun_out/r1h
for cfg in "16 8 0" "1 65 0" "16 8 1"; do
  set -- $cfg
  echo "trig=$1 keep=$2 diag=$3" >> gpurun_out/r1h/sweep.log
  PT_DIAG=$3 PT_MARCH_TRIGGER=$1 PT_MARCH_KEEP=$2 timeout -k 10 120 python scripts/phase_profile.py 16 >> gpurun_out/r1h/sweep.log 2>&1
done
