# r03i: GPT-2 block with the chunked FFN hidden layout (reduced, then GPT-2 width with a 160 GB
# mask cache), ResNet-20 with bootstrap-only lockstep (MHE_RESNET_LOCKSTEP=2) vs 4 streams, and the
# ModUp column pass compiled for 2 waves/SIMD (no spills) vs 3.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i
mkdir -p $O
bash scripts/gpu_sq.sh || exit $?
timeout -k 10 300 ./build/seal_batch_test 13 > $O/seal_batch13.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mixed or reference_chains or variants or hmult_small" > $O/pytest_mixed.log 2>&1 || exit $?
timeout -k 10 300 ./build/gpt2_block_test tests/golden/gpt2_block > $O/gpt2_small.log 2>&1 || exit $?
for v in 2 0 2; do
  MHE_RESNET_LOCKSTEP=$v MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 600 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet_ls${v}_$(date +%s).log 2>&1 || exit $?
done
for lib in mocc2 dpf2 cur mocc2 dpf2 cur; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 5 --warmup 2 > $O/hm_${lib}_$(date +%s).json 2> /dev/null || exit $?
done
unset MHE_LIB_PATH
FX=$(mktemp -d /tmp/gpt2fx.XXXXXX)
python3 tests/golden/gpt2_block/make_fixture.py --full "$FX" > $O/gpt2_full_fixture.log 2>&1 || exit $?
MHE_VEC_CACHE_GB=100 MHE_BLOCK_VERBOSE=1 timeout -k 10 500 ./build/gpt2_block_test "$FX" block > $O/gpt2_full.log 2>&1
rc=$?
rm -rf "$FX"
exit $rc
