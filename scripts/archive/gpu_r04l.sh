# r04l: hoisted rotations: batch parity, then the 8x7 / 1x7 microbenchmark at 31 limbs (hoisted with
# prefetch depth 3 / 2 / 1, classic) and kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04l
rm -f gpurun_out/r04l/ub.jsonl
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -k rotate --timeout 380 --timeout-method thread > gpurun_out/r04l/batch.log 2>&1 || exit $?
for b in 8x7 1x7; do
  for h in 1 0; do
    MHE_KS_HOIST=$h timeout -k 10 200 python scripts/ubench_ops.py --ops bsgs --bsgs $b --limbs 31 --reps 5 >> gpurun_out/r04l/ub.jsonl 2>> gpurun_out/r04l/ub.err || exit $?
  done
  for v in none; do [ "$v" = none ] && continue
    MHE_LIB_PATH=build/var/$v/libmhe.so timeout -k 10 200 python scripts/ubench_ops.py --ops bsgs --bsgs $b --limbs 31 --reps 5 >> gpurun_out/r04l/ub.jsonl 2>> gpurun_out/r04l/ub.err || exit $?
  done
done
d="$R/gpurun_out/r04l/prof"
mkdir -p "$d"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o ub --output-format csv -- python3 "$R/scripts/ubench_ops.py" --ops bsgs --bsgs 8x7 --limbs 31 --reps 5 > "$d/ub.log" 2>&1 || exit $?
find "$d" -name "*kernel_trace*" -delete
