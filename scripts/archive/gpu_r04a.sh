# r04a: the bench's own timed path vs the oracle, batch-entry overlap checks, SEAL surface tests, bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bench_path.py tests/test_gpu_batch.py tests/test_seal_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_pytest.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench.log 2>&1 || exit $?
