# r03y: ModUp column pass with the group's twiddles staged in LDS (build/var/twl) and with only the
# unpacked-store addressing fix (build/var/twl0, -DMHE_MODUP_TWG=0) vs HEAD; parity with twl first.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03y
mkdir -p $O
MHE_LIB_PATH=$PWD/build/var/twl/libmhe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_twl.log 2>&1 || exit $?
for lib in cur twl twl0 cur twl twl0; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 python scripts/ubench_ops.py --ops ks,ks4,rot4,hmult >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
  timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > $O/hm_${lib}_$(date +%s).json 2>> $O/err.log || exit $?
done
unset MHE_LIB_PATH
for lib in cur twl; do
  if [ $lib = twl ]; then export MHE_LIB_PATH="$PWD/build/var/twl/libmhe.so"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_$lib" -o p --output-format csv -- python3 scripts/ubench_ops.py --ops ks4 --reps 20 > /dev/null 2>> $O/ops.err || exit $?
done
