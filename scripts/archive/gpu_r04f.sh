# r04f: FiberBatch with coalesced elementwise launches: correctness (seal_batch_test), then ResNet-20
# 8-image batches: 4 streams vs fibers (threads x fibers 2x4, 4x2, 1x8), then the trace parity
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -k seal_surface --timeout 280 --timeout-method thread > gpurun_out/r04f/seal_batch.log 2>&1 || exit $?
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "streams4 4 1" "f4x2 2 4" "f2x4 4 2" "f8x1 1 8"; do
  set -- $v
  MHE_RESNET_FIBERS=$3 MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 300 ./build/resnet_test $P $C 8 20 $2 > gpurun_out/r04f/$1.log 2>&1 || exit $?
done
bash scripts/gpu_r04c.sh
