# r03q: the special limbs' inverse row pass inside the fused key MAC (MHE_KS_INV_FUSED): parity
# (engine, batched entry points, trace), per-op A/B with the separate k_inv_row, ResNet-20 timing
# and one steady-state image's kernel / launch counts.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_trace_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for f in 0 1 0 1; do
  MHE_KS_INV_FUSED=$f timeout -k 10 200 python scripts/ubench_ops.py --ops ks,ks4,rot4,hmult >> $O/ops_f$f.jsonl 2>> $O/ops.err || exit $?
done
for f in 0 1; do
  MHE_KS_INV_FUSED=$f timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > $O/hm_f$f.json 2>> $O/ops.err || exit $?
done
timeout -k 10 400 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet4.log 2>&1 || exit $?
rm -rf gpurun_out/prof_rn1 gpurun_out/prof_rn2
bash scripts/gpu_prof_resnet_diff.sh || exit $?
python3 scripts/kstats.py diff gpurun_out/prof_rn1/rn_kernel_stats.csv gpurun_out/prof_rn2/rn_kernel_stats.csv > $O/resnet20_per_image_kernels.txt
