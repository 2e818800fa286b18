# r03f: row-MAC kernel variants (MHE_KS_EB: 0 = E8 + transpose back, 2 = E4 @3 waves, 4 = E4 @4
# waves, 3 = E8 MAC-in-place @2 waves): parity on the key-switch tests, then HMult bench A/B
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f
mkdir -p $O
for eb in 2 4 3; do
  MHE_KS_EB=$eb timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hmult or switch or rotate or galois or relin or key" > $O/pytest_eb$eb.log 2>&1 || exit $?
done
for eb in 0 2 4 3 0 2; do
  MHE_KS_EB=$eb timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 5 --warmup 2 > $O/hm_eb$eb.json 2> $O/hm_eb$eb.err || exit $?
  cp $O/hm_eb$eb.json $O/hm_eb${eb}_$(date +%s).json
done
for eb in 0 2; do
  MHE_KS_EB=$eb timeout -k 10 300 ./build/boot_test 14 2 > $O/boot_eb$eb.log 2>&1 || exit $?
done
