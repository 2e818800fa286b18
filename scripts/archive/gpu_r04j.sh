# r04j: hoisted rotations: ResNet-20 8-image fiber batch (2 threads x 4 fibers) with / without
# hoisting, then rocprofv3 kernel stats of a 2-image single-thread run in each mode
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04j
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "hoist1 1" "hoist0 0"; do
  set -- $v
  MHE_KS_HOIST=$2 MHE_RESNET_FIBERS=4 timeout -k 10 300 ./build/resnet_test $P $C 8 20 2 > gpurun_out/r04j/$1.log 2>&1 || exit $?
done
for v in "hoist1 1" "hoist0 0"; do
  set -- $v
  d="$R/gpurun_out/r04j/prof_$1"
  mkdir -p "$d"
  MHE_KS_HOIST=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o rn --output-format csv -- "$R/build/resnet_test" $P $C 2 20 1 > "$d/rn.log" 2>&1 || exit $?
  find "$d" -name "*kernel_trace*" -delete
done
