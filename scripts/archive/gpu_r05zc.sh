# r05zc: A/B of the encoder's pinned upload ring (main: 64 slots, build/vx/base: 8) on the ResNet-20
# 3 x 8 batch, alternated twice (libmhe_seal loads libmhe.so through its runpath: LD_LIBRARY_PATH
# swaps it)
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05zc_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for rep in 1 2; do
  for lib in main base; do
    if [ $lib = main ]; then LD=$GRAFT_REPO_ROOT/fhe-gpt-2_amd; else LD=$GRAFT_REPO_ROOT/build/vx/$lib; fi
    LD_LIBRARY_PATH=$LD MHE_RESNET_FIBERS=8 timeout -k 10 400 ./build/resnet_test $P $C 24 20 3 > $D/resnet_${lib}_$rep.log 2>&1; rc=$?
    echo "$lib $rep rc=$rc $(grep '^batch:' $D/resnet_${lib}_$rep.log) $(tail -1 $D/resnet_${lib}_$rep.log)" | tee -a $D/summary.txt
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
done
