# Per-image ResNet-20 kernel stats: rocprofv3 stats of a 1-image and a 2-image run (same setup);
# their difference is one steady-state image (scripts/kstats.py diff).
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_rn1 gpurun_out/prof_rn2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_rn1" -o rn --output-format csv -- "$R/build/resnet_test" "$R/tests/golden/resnet/resnet20_params.bin" "$R/tests/golden/comp" 1 20 0 > gpurun_out/prof_rn1/rn.log 2>&1
rc=$?
find gpurun_out/prof_rn1 -name "*kernel_trace*" -delete
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_rn2" -o rn --output-format csv -- "$R/build/resnet_test" "$R/tests/golden/resnet/resnet20_params.bin" "$R/tests/golden/comp" 2 20 0 > gpurun_out/prof_rn2/rn.log 2>&1
rc=$?
find gpurun_out/prof_rn2 -name "*kernel_trace*" -delete
exit $rc
