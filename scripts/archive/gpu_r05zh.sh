# r05zh: no zero fill before a full-slot encode (main) vs always (build/vx/base): parity subset,
# then the ResNet-20 3 x 8 batch alternated twice (libmhe_seal loads libmhe.so through its runpath: LD_LIBRARY_PATH
# swaps it)
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05zh_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_seal_api.py tests/test_gpt2.py > $D/parity.log 2>&1; rc=$?
echo "parity rc=$rc"; tail -1 $D/parity.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in main base; do
    if [ $lib = main ]; then LD=$GRAFT_REPO_ROOT/fhe-gpt-2_amd; else LD=$GRAFT_REPO_ROOT/build/vx/$lib; fi
    LD_LIBRARY_PATH=$LD MHE_RESNET_FIBERS=8 timeout -k 10 400 ./build/resnet_test $P $C 24 20 3 > $D/resnet_${lib}_$rep.log 2>&1; rc=$?
    echo "$lib $rep rc=$rc $(grep '^batch:' $D/resnet_${lib}_$rep.log) $(tail -1 $D/resnet_${lib}_$rep.log)" | tee -a $D/summary.txt
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
done
