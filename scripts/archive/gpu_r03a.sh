# r03a: batched-launch parity + the existing parity file, then a kernel trace of boot_test
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1 || exit $?
bash scripts/gpu_boot_trace.sh
