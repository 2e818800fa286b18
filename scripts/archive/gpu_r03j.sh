# r03j: row-pass epilogue prefetch (MHE_ROW_PRE) -- parity file, per-op A/B at ResNet levels against
# the build without it (build/var/base), HMult leg, ResNet-20 4 images x 4 threads with
# MHE_RESNET_LOCKSTEP 0 (independent streams) / 2 (bootstrap-only merge) / 1 (every key switch merged).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || exit $?
for lib in base cur base cur; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 python scripts/ubench_ops.py >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
done
unset MHE_LIB_PATH
timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > $O/hm.json 2> $O/hm.err || exit $?
for v in 0 2 1; do
  MHE_RESNET_LOCKSTEP=$v MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 400 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet_ls$v.log 2>&1 || exit $?
done
