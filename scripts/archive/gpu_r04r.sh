# r04r: round-4 HEAD: rotation / trace / timed-path parity, the BSGS microbenchmark, the default bench
# (HMult + ResNet-20 legs, CPU baseline) and the HMult leg's rocprofv3 kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04r
rm -f gpurun_out/r04r/ub.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_trace_parity.py tests/test_bench_path.py -m gpu -x -q --timeout 580 --timeout-method thread > gpurun_out/r04r/tests.log 2>&1 || exit $?
for b in 8x7 1x7; do
  timeout -k 10 200 python scripts/ubench_ops.py --ops bsgs --bsgs $b --limbs 31 --reps 5 >> gpurun_out/r04r/ub.jsonl 2>> gpurun_out/r04r/ub.err || exit $?
done
timeout -k 10 600 python bench.py > gpurun_out/r04r/bench.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r04r/prof" -o r04r --output-format csv -- python3 "$R/bench.py" --no-cpu --resnet-images 0 --streams 1 --steps 3 --warmup 1 > gpurun_out/r04r/prof.log 2>&1 || exit $?
find gpurun_out/r04r/prof -name "*kernel_trace*" -delete
