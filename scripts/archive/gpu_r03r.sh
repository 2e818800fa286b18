# r03r: ResNet-20 4 images with the batched callers x MHE_RESNET_LOCKSTEP 0 / 1 / 2; the fused MAC
# with the intermediate prefetched two digits ahead (build/var/dpf2) on both legs; SQ counters of
# the C2 key-switch kernels (8 HMults sharing the relin key).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03r
mkdir -p $O
for v in 0 1 2 0 1 2; do
  MHE_RESNET_LOCKSTEP=$v MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 400 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet_ls${v}_$(date +%s).log 2>&1 || exit $?
done
for lib in cur dpf2 cur dpf2; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 python scripts/ubench_ops.py --ops ks,ks4,ks4s,rot4,hmult >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
  timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > $O/hm_${lib}_$(date +%s).json 2>> $O/ops.err || exit $?
done
unset MHE_LIB_PATH
bash scripts/gpu_sq.sh > $O/sq.log 2>&1 || exit $?
cp gpurun_out/sq_counters.json $O/ 2>/dev/null
exit 0
