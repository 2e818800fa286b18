# HMult leg: independent HMults per step (batch) x streams, same box
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bt
for cfg in "8 4" "16 4" "32 4" "16 3" "8 4" "32 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --batch $1 --streams $2 > gpurun_out/bt/b$1_s$2.json 2>/dev/null || exit $?
  echo "batch=$1 streams=$2 $(grep -o '"value": [0-9.]*' gpurun_out/bt/b$1_s$2.json) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bt/b$1_s$2.json)" >> gpurun_out/bt/summary.txt
done
