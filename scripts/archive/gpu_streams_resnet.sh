set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -x --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
timeout -k 10 300 ./build/resnet_test $P $C 8 20 8 > gpurun_out/rn_s8.log 2>&1 || exit $?
timeout -k 10 300 ./build/resnet_test $P $C 8 20 4 > gpurun_out/rn_s4.log 2>&1 || exit $?
