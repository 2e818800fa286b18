# Inverse column pass fused into the ModDown / rescale lift column pass: parity, seal tests,
# then the ResNet leg A/B via MHE_ICOL_FUSED.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_seal_api.py -m gpu -q -x --timeout 500 --timeout-method thread > gpurun_out/icol_tests.log 2>&1 || exit $?
: > gpurun_out/icol_summary.txt
for v in ${ICOL_VARIANTS:-1 0 1 0}; do
  MHE_ICOL_FUSED=$v timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/icol_$v.log 2>&1 || exit $?
  echo "fused=$v $(grep -o '"sec_per_image_1stream": [0-9.]*\|"images_per_s": [0-9.]*' gpurun_out/icol_$v.log | tr '\n' ' ')" >> gpurun_out/icol_summary.txt
done
