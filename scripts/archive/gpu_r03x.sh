# r03x: 16 HMults per key switch (build/var/maxb16, -DMHE_MAXB=16) vs 8 on the C2 HMult leg, same box;
# parity file with the 16-entry build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x
mkdir -p $O
MHE_LIB_PATH=$PWD/build/var/maxb16/libmhe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_maxb16.log 2>&1 || exit $?
for lib in cur maxb16 cur maxb16; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; G=8; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; G=16; fi
  timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 --hmult-group $G > $O/hm_${lib}_$(date +%s).json 2>> $O/err.log || exit $?
done
export MHE_LIB_PATH=$PWD/build/var/maxb16/libmhe.so
timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 --hmult-group 16 --batch 64 > $O/hm_maxb16_b64.json 2>> $O/err.log || exit $?
