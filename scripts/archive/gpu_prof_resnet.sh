# One ResNet-20 image under rocprofv3 kernel-trace stats (current code), summary + launch counts.
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_resnet
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_resnet" -o rn --output-format csv -- "$R/build/resnet_test" "$R/tests/golden/resnet/resnet20_params.bin" "$R/tests/golden/comp" 1 20 1 > gpurun_out/prof_resnet/rn.log 2>&1
rc=$?
find gpurun_out/prof_resnet -name "*kernel_trace*" -delete
exit $rc
