# Round profiles: rocprofv3 kernel-trace stats of the HMult bench (single stream, so per-launch
# durations compare with the bench's own HIP events) and of one ResNet-20 image (resnet_test).
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/prof_resnet
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o hmult --output-format csv -- python3 "$R/bench.py" --no-cpu --streams 1 --steps 3 --warmup 1 --resnet-images 0 > gpurun_out/prof/hmult.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_resnet" -o resnet --output-format csv -- "$R/build/resnet_test" "$R/tests/golden/resnet/resnet20_params.bin" "$R/tests/golden/comp" 1 20 1 > gpurun_out/prof_resnet/resnet.log 2>&1 || exit $?
