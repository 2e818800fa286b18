# r03zm: integer / MIX ModUp column pass at 2 waves/SIMD (no spills; build/var/mix) vs HEAD on the
# GPT-2 chain (its special prime >= 2^51 takes the MIX kernel): GPU parity files with mix, then the
# reduced GPT-2 block and the full-width block, each both ways.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03zm
mkdir -p $O
[ -n "${SKIP_PYTEST:-}" ] || MHE_LIB_PATH=$PWD/build/var/mix/libmhe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_mix.log 2>&1 || exit $?
for v in cur mix cur mix; do
  if [ $v = cur ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH="$PWD/build/var/mix"; fi
  t0=$(date +%s%N); timeout -k 10 300 ./build/gpt2_block_test tests/golden/gpt2_block > $O/small_$v.$t0.log 2>&1 || exit $?; echo "$v $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $O/small_times.txt
done
for v in cur mix; do
  if [ $v = cur ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH="$PWD/build/var/mix"; fi
  FX=$(mktemp -d /tmp/gpt2fx.XXXXXX)
  python3 tests/golden/gpt2_block/make_fixture.py --full "$FX" > $O/fixture.log 2>&1 || exit $?
  MHE_VEC_CACHE_GB=100 MHE_BLOCK_VERBOSE=1 timeout -k 10 300 ./build/gpt2_block_test "$FX" block > $O/full_$v.log 2>&1
  rc=$?; rm -rf "$FX"; [ $rc -eq 0 ] || exit $rc
done
