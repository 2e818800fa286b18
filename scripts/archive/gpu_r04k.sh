# r04k: hoisted rotations microbenchmark: 8 inputs x 7 rotations (shared keys) and 1 x 7 at 31 and 19
# limbs, with / without hoisting, then kernel stats of the hoisted 8x7 at 31 limbs
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04k
export TMPDIR=/tmp
for L in 31 19; do for b in 8x7 1x7; do for h in 1 0; do
  MHE_KS_HOIST=$h timeout -k 10 200 python scripts/ubench_ops.py --ops bsgs --bsgs $b --limbs $L --reps 5 >> gpurun_out/r04k/ub.jsonl 2>> gpurun_out/r04k/ub.err || exit $?
done; done; done
d="$R/gpurun_out/r04k/prof"
mkdir -p "$d"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o ub --output-format csv -- python3 "$R/scripts/ubench_ops.py" --ops bsgs --bsgs 8x7 --limbs 31 --reps 5 > "$d/ub.log" 2>&1 || exit $?
find "$d" -name "*kernel_trace*" -delete
