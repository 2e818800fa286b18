# r03d: engine A/B (LDS-only barriers in the ModUp column pass + 2^52-offset conversions vs the
# batching commit), then bootstrapping / ResNet accuracy with the Remez-generated EvalMod cosine
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_ab_r03.sh > gpurun_out/ab_summary.txt 2>&1 || exit $?
for ln in 14 13 12; do timeout -k 10 300 ./build/boot_test $ln 2 > gpurun_out/r03d_boot$ln.log 2>&1 || exit $?; done
timeout -k 10 600 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > gpurun_out/r03d_resnet.log 2>&1 || exit $?
