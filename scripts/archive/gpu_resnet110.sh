# ResNet-110 (config C4's network) and serialization checks on one GPU
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_serialize.py tests/test_seal_api.py -m gpu -v -x --timeout 600 --timeout-method thread -s > gpurun_out/r110_test.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu --steps 3 --warmup 1 --resnet-layers 110 --resnet-images 4 --resnet-streams 4 > gpurun_out/r110_bench.log 2>&1 || exit $?
