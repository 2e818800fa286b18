# r03b: batched-launch parity, parity file, SEAL-surface tests, then ResNet-20 timing and a boot trace
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_seal_api.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1 || exit $?
timeout -k 10 300 ./build/boot_test 14 3 > gpurun_out/r03b_boot.log 2>&1 || exit $?
timeout -k 10 600 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > gpurun_out/r03b_resnet.log 2>&1 || exit $?
bash scripts/gpu_boot_trace.sh
