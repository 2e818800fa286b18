# r03s: moves instead of device copies for dead ciphertexts in the callers (conv, BN, ReLU, add,
# downsampling, pooling, FC, BSGS giant sums, EvalMod heap) -- parity / trace / ResNet tests, ResNet
# timing and launch counts; C2 HMult leg with SEAL's key layout vs the prepared 48-bit key now that
# 8 HMults share the key stream.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_trace_parity.py tests/test_seal_api.py -m gpu -x -q --timeout 600 --timeout-method thread -k "trace or relu or resnet20_end or stage_levels or bootstrapping or cnn_layers" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet4.log 2>&1 || exit $?
for kf in seal prepared seal prepared; do
  timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 --key-format $kf > $O/hm_${kf}_$(date +%s).json 2>> $O/err.log || exit $?
done
rm -rf gpurun_out/prof_rn1 gpurun_out/prof_rn2
bash scripts/gpu_prof_resnet_diff.sh || exit $?
python3 scripts/kstats.py diff gpurun_out/prof_rn1/rn_kernel_stats.csv gpurun_out/prof_rn2/rn_kernel_stats.csv > $O/resnet20_per_image_kernels.txt
