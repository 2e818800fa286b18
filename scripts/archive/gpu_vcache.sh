# Static-vector plaintext cache: seal/cnn/resnet tests, then the ResNet leg A/B via MHE_VEC_CACHE_GB.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_seal_api.py tests/test_resnet_keys.py -m gpu -q -x --timeout 500 --timeout-method thread > gpurun_out/vc_tests.log 2>&1 || exit $?
: > gpurun_out/vc_summary.txt
for v in ${VC_VARIANTS:-48 0 48 0}; do
  MHE_VEC_CACHE_GB=$v timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/vc_$v.log 2>&1 || exit $?
  echo "cache=$v $(grep -o '"sec_per_image_1stream": [0-9.]*\|"images_per_s": [0-9.]*' gpurun_out/vc_$v.log | tr '\n' ' ')" >> gpurun_out/vc_summary.txt
done
