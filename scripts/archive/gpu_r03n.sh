# r03n: (1) conflict-free twiddle LDS slots in the fused key MAC (build/var/twz): parity + per-op A/B;
# (2) does the Infinity Cache keep the ModUp intermediate between the two key-switch kernels when
# it is not stored non-temporally?  Output-prime chunks (MHE_KS_FCHUNK) with MHE_NT = 0 (all
# temporal) and MHE_NT = 2 (only the key loads non-temporal), at L = 31 and on the C2 HMult leg.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03n
mkdir -p $O
MHE_LIB_PATH=$PWD/build/var/twz/libmhe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity_twz.log 2>&1 || exit $?
for lib in cur twz cur twz; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 python scripts/ubench_ops.py --ops ks,ks4,ks4s,rot4,hmult >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
done
for lib in cur nt0 nt2; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  for fc in 0 4 8 16; do
    MHE_KS_FCHUNK=$fc timeout -k 10 200 python scripts/ubench_ops.py --ops ks,ks4s --reps 30 | sed "s/}/, \"fchunk\": $fc, \"v\": \"$lib\"}/" >> $O/sweep.jsonl 2>> $O/ops.err || exit $?
  done
  for fc in 0 3 5 9; do
    MHE_KS_FCHUNK=$fc timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 5 --warmup 2 > $O/hm_${lib}_fc$fc.json 2>> $O/ops.err || exit $?
  done
done
