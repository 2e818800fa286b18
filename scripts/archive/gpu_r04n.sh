# r04n: hoisted rotations end to end: trace parity (conv / BN / ReLU, bootstrap, layers), the seal batch
# tests, then ResNet-20 8-image fiber batches (2 threads x 4 fibers) with / without hoisting, twice
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04n
timeout -k 10 500 python -u -m pytest tests/test_trace_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 480 --timeout-method thread > gpurun_out/r04n/tests.log 2>&1 || exit $?
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "h1a 1" "h0a 0" "h1b 1" "h0b 0"; do
  set -- $v
  MHE_KS_HOIST=$2 MHE_RESNET_FIBERS=4 timeout -k 10 300 ./build/resnet_test $P $C 8 20 2 > gpurun_out/r04n/$1.log 2>&1 || exit $?
done
# SQ counters of the shared-key hoisted MAC (8 x 7 rotations, 31 limbs)
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/r04n/pmc"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex "hoist" -d "$OUT" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/ubench_ops.py" --ops bsgs --bsgs 8x7 --limbs 31 --reps 1 > "$OUT/p.log" 2>&1 || exit $?
