# HMult bench with the nontemporal-access variants of libmhe (exp/libmhe_nt*.so) vs the default.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${NT_VARIANTS:-base 1 6 7 base}; do
  if [ "$v" = base ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$GRAFT_REPO_ROOT/exp/libmhe_$v.so"; fi
  timeout -k 10 200 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > gpurun_out/nt_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/nt_$v.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/nt_$v.log)" >> gpurun_out/nt_summary.txt
done
