# Packed (48-bit) ModUp intermediate: parity at C2 size, then HMult A/B via MHE_KS_PACK.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pack_parity.log 2>&1 || exit $?
: > gpurun_out/pack_summary.txt
for v in ${PACK_VARIANTS:-1 0 1 0}; do
  MHE_KS_PACK=$v timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 --resnet-images 0 > gpurun_out/pack_$v.log 2>&1 || exit $?
  echo "pack=$v $(grep -o '"value": [0-9.]*\|"achieved": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/pack_$v.log | tr '\n' ' ')" >> gpurun_out/pack_summary.txt
done
