# r03g: ModUp output-prime chunks sized for the 256 MB Infinity Cache now that a key switch covers
# 8 HMults (MHE_KS_FCHUNK), with the intermediate streamed non-temporally (current build, MHE_NT=5),
# cached (MHE_NT=0) or NT stores + cached loads (MHE_NT=1); parity of each library first.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g
mkdir -p $O
for lib in cur nt0 nt1; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  MHE_KS_FCHUNK=9 timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 240 --timeout-method thread -k "hmult or switch" > $O/pytest_$lib.log 2>&1 || exit $?
  for ch in 0 5 9 15; do
    MHE_KS_FCHUNK=$ch timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 5 --warmup 2 > $O/hm_${lib}_c$ch.json 2> $O/hm_${lib}_c$ch.err || exit $?
  done
done
# the GPT-2-width block under rocprofv3 --kernel-trace --stats (kernel time vs wall, launches)
unset MHE_LIB_PATH
FX=$(mktemp -d /tmp/gpt2fx.XXXXXX)
python3 tests/golden/gpt2_block/make_fixture.py --full "$FX" > $O/gpt2_fixture.log 2>&1 || exit $?
export TMPDIR=/tmp
MHE_BLOCK_VERBOSE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_gpt2" -o gpt2 --output-format csv -- ./build/gpt2_block_test "$FX" block > $O/gpt2_full_prof.log 2>&1
rc=$?
rm -rf "$FX"
find $O/prof_gpt2 -name "*kernel_trace*" -delete
exit $rc
