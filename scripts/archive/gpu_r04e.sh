# r04e: KS parity after the centred 48-bit ModUp intermediate (FP path), the bench path, then bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04e_parity.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04e_bench.log 2>&1 || exit $?
