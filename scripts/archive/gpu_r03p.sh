# r03p: (1) the ReLU polynomial (seal/comp.cpp) and the EvalMod heap polynomial (seal/boot.cpp)
# with each depth's products / rescales batched: trace parity (op by op vs the oracle), approximate
# ReLU, bootstrapping (boot_test also compares batched vs one-by-one launches word for word) and
# ResNet-20 end-to-end tests, the reference stage log, ResNet-20 timing and one steady-state image's
# kernel / launch counts. 
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_trace_parity.py tests/test_seal_api.py -m gpu -x -v --timeout 600 --timeout-method thread -k "trace or relu or resnet20_end or stage_levels or bootstrapping" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet4.log 2>&1 || exit $?
rm -rf gpurun_out/prof_rn1 gpurun_out/prof_rn2
bash scripts/gpu_prof_resnet_diff.sh || exit $?
python3 scripts/kstats.py diff gpurun_out/prof_rn1/rn_kernel_stats.csv gpurun_out/prof_rn2/rn_kernel_stats.csv > $O/resnet20_per_image_kernels.txt
