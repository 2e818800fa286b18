# r03e: batched HMult (shared relin key stream) parity + bench A/B, seal-surface batches, seeded
# serialization, the GPT-2 block after the matmul rework, Remez bootstrapping accuracy, ResNet-20.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03e
O=gpurun_out/r03e
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_serialize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_batch.log 2>&1 || exit $?
for v in "8 1" "8 0" "1 1" "8 1"; do
  set -- $v
  MHE_KS_SHARE=$2 timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 5 --warmup 2 --hmult-group $1 > $O/hm_g$1_s$2.json 2> $O/hm_g$1_s$2.err || exit $?
done
timeout -k 10 300 ./build/gpt2_block_test tests/golden/gpt2_block > $O/gpt2_small.log 2>&1 || exit $?
for ln in 14 13 12; do timeout -k 10 300 ./build/boot_test $ln 2 > $O/boot$ln.log 2>&1 || exit $?; done
timeout -k 10 600 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet.log 2>&1 || exit $?
