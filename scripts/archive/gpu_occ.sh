# Fused-MAC occupancy variants (exp/libmhe_<v>.so, MHE_KS_XCH/OCC/DPF builds): C2 parity, then HMult A/B.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/occ_summary.txt
for v in ${OCC_VARIANTS:-o3d0 o3d1}; do
  MHE_LIB_PATH="$GRAFT_REPO_ROOT/exp/libmhe_$v.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > gpurun_out/occ_parity_$v.log 2>&1 || exit $?
done
for v in ${OCC_RUNS:-base o3d0 o3d1 base o3d0 o3d1}; do
  if [ "$v" = base ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$GRAFT_REPO_ROOT/exp/libmhe_$v.so"; fi
  timeout -k 10 200 python bench.py --no-cpu --resnet-images 0 --steps 20 --warmup 3 > gpurun_out/occ_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/occ_$v.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/occ_$v.log)" >> gpurun_out/occ_summary.txt
done
