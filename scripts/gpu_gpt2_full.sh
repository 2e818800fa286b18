# C5 at GPT-2 width: the reduced block first (refactor check, 1e-3), then the whole block at
# T 128, d 768, 12 heads, d_ff 3072 against the full-width restatement regenerated from its seed.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./build/gpt2_block_test tests/golden/gpt2_block > gpurun_out/gpt2_small.log 2>&1 || exit $?
FX=$(mktemp -d /tmp/gpt2fx.XXXXXX)
python3 tests/golden/gpt2_block/make_fixture.py --full "$FX" > gpurun_out/gpt2_full_fixture.log 2>&1 || exit $?
MHE_VEC_CACHE_GB=${VEC_CACHE_GB:-100} MHE_BLOCK_VERBOSE=1 timeout -k 10 ${FULL_LIMIT:-1000} ./build/gpt2_block_test "$FX" block > gpurun_out/gpt2_full.log 2>&1
rc=$?
rm -rf "$FX"
exit $rc
