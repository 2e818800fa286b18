# r03h: seal batches incl. the Lockstep group (seal_batch_test), the reduced GPT-2 block after the
# operand drop, then the GPT-2-width block (verbose stage times) and ResNet-20 with and without
# MHE_RESNET_LOCKSTEP.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h
mkdir -p $O
for ln in 13 16; do timeout -k 10 300 ./build/seal_batch_test $ln > $O/seal_batch$ln.log 2>&1 || exit $?; done
timeout -k 10 300 ./build/gpt2_block_test tests/golden/gpt2_block > $O/gpt2_small.log 2>&1 || exit $?
for v in 1 0; do
  MHE_RESNET_LOCKSTEP=$v MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 600 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet_ls$v.log 2>&1 || exit $?
done
FX=$(mktemp -d /tmp/gpt2fx.XXXXXX)
python3 tests/golden/gpt2_block/make_fixture.py --full "$FX" > $O/gpt2_full_fixture.log 2>&1 || exit $?
MHE_BLOCK_VERBOSE=1 timeout -k 10 700 ./build/gpt2_block_test "$FX" block > $O/gpt2_full.log 2>&1
rc=$?
rm -rf "$FX"
exit $rc
