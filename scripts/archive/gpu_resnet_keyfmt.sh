# ResNet with prepared keys: key export/import + ResNet-20 tests, then a bench A/B of the ResNet leg
# (MHE_KEY_PREPARE=0 vs default) and of the fused MAC's key prefetch (MHE_KS_KPF=1) on the HMult leg
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rk
timeout -k 10 600 python -u -m pytest tests/test_resnet_keys.py tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread \
  -k "exported_keys or resnet20_end_to_end or prepared" > gpurun_out/rk/pytest.log 2>&1 || exit $?
B="timeout -k 10 400 python bench.py --no-cpu --steps 10 --resnet-images 4"
MHE_KEY_PREPARE=0 $B > gpurun_out/rk/bench_seal.json 2>gpurun_out/rk/bench_seal.err || exit $?
$B > gpurun_out/rk/bench_prep.json 2>gpurun_out/rk/bench_prep.err || exit $?
MHE_KS_KPF=1 timeout -k 10 300 python bench.py --no-cpu --steps 20 --resnet-images 0 > gpurun_out/rk/bench_kpf.json 2>gpurun_out/rk/bench_kpf.err || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 20 --resnet-images 0 > gpurun_out/rk/bench_nokpf.json 2>gpurun_out/rk/bench_nokpf.err || exit $?
