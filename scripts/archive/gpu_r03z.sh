# r03z: k_icol_lift with the group's forward column twiddles staged in LDS (build/var/icol) vs HEAD
# 418597f; parity with icol first; rescale / key-switch microbenchmarks at 31 limbs, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03z
mkdir -p $O
MHE_LIB_PATH=$PWD/build/var/icol/libmhe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_icol.log 2>&1 || exit $?
for lib in cur icol cur icol; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 python scripts/ubench_ops.py --ops rescale,rescale4,ks4,hmult >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
done
for lib in cur icol; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_$lib" -o p --output-format csv -- python3 scripts/ubench_ops.py --ops rescale4,ks4 --reps 20 > /dev/null 2>> $O/ops.err || exit $?
done
