# r04o: hoisted rotations: rotate parity, trace parity, microbenchmark, ResNet-20 8-image fiber batch
# with / without hoisting (twice each)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04o
rm -f gpurun_out/r04o/ub.jsonl
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch.py tests/test_trace_parity.py -m gpu -x -q --timeout 480 --timeout-method thread > gpurun_out/r04o/tests.log 2>&1 || exit $?
for b in 8x7 1x7; do for h in 1 0; do
  MHE_KS_HOIST=$h timeout -k 10 200 python scripts/ubench_ops.py --ops bsgs --bsgs $b --limbs 31 --reps 5 >> gpurun_out/r04o/ub.jsonl 2>> gpurun_out/r04o/ub.err || exit $?
done; done
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "h1a 1" "h0a 0" "h1b 1" "h0b 0"; do
  set -- $v
  MHE_KS_HOIST=$2 MHE_RESNET_FIBERS=4 timeout -k 10 300 ./build/resnet_test $P $C 8 20 2 > gpurun_out/r04o/$1.log 2>&1 || exit $?
done
