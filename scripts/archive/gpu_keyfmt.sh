# Prepared-key format: parity subset, then an alternating A/B of bench.py's HMult leg (seal vs prepared key);
# then ModUp chunks small enough for the Infinity Cache, with cached (MHE_NT=0) intermediate accesses
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kf
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "prepared or hmult or switch_key or rotate or variants" > gpurun_out/kf/pytest.log 2>&1 || exit $?
B="timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 20"
for i in 1 2; do
  for f in seal prepared; do
    $B --key-format $f > gpurun_out/kf/bench_${f}_$i.json 2>gpurun_out/kf/bench_${f}_$i.err || exit $?
  done
done
for ch in 0 8 15; do
  MHE_LIB_PATH=$GRAFT_REPO_ROOT/exp/libmhe_nt0.so MHE_KS_FCHUNK=$ch $B > gpurun_out/kf/bench_nt0_fc$ch.json 2>gpurun_out/kf/bench_nt0_fc$ch.err || exit $?
  MHE_KS_FCHUNK=$ch $B > gpurun_out/kf/bench_nt5_fc$ch.json 2>gpurun_out/kf/bench_nt5_fc$ch.err || exit $?
done
