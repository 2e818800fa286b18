# A/B of libmhe_seal variants (exp/libmhe_seal_<v>.so vs the in-tree one) on the ResNet leg.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab_summary.txt
for v in ${AB_VARIANTS:-new old new old}; do
  if [ "$v" = new ]; then unset MHE_SEAL_LIB_PATH; else export MHE_SEAL_LIB_PATH="$GRAFT_REPO_ROOT/exp/libmhe_seal_$v.so"; fi
  timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/ab_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"sec_per_image_1stream": [0-9.]*\|"images_per_s": [0-9.]*' gpurun_out/ab_$v.log | tr '\n' ' ')" >> gpurun_out/ab_summary.txt
done
