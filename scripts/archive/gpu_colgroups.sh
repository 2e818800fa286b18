# ModUp column pass: output-prime groups per digit (MHE_KS_COLGROUPS), same box, HMult leg
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cg
for g in 9 12 15 6 23 9; do
  MHE_KS_COLGROUPS=$g timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 > gpurun_out/cg/g$g.json 2>/dev/null || exit $?
  echo "colgroups=$g $(grep -o '"value": [0-9.]*' gpurun_out/cg/g$g.json) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/cg/g$g.json) $(grep -o '"modup_col_avg_launch_us": [0-9.]*' gpurun_out/cg/g$g.json)" >> gpurun_out/cg/summary.txt
done
