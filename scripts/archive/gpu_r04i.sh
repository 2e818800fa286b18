# r04i: hoisted rotations (csrc/hoist.h): batched-rotation parity vs the oracle incl. zero-coefficient
# inputs (classic fallback), the caller-sequence traces (conv/BN/ReLU, bootstrap, layers), then
# ResNet-20 8-image batches (2 threads x 4 fibers) with and without hoisting on the same box
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04i
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -v --timeout 380 --timeout-method thread > gpurun_out/r04i/batch.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_trace_parity.py -m gpu -x -v --timeout 480 --timeout-method thread > gpurun_out/r04i/trace.log 2>&1 || exit $?
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "hoist1 1" "hoist0 0" "hoist1b 1"; do
  set -- $v
  MHE_KS_HOIST=$2 MHE_RESNET_FIBERS=4 timeout -k 10 300 ./build/resnet_test $P $C 8 20 2 > gpurun_out/r04i/$1.log 2>&1 || exit $?
done
