# r05g: stream pool (threads that exit hand their stream + scratch to the next thread); ResNet-20
# batch shapes around 3 x 8; fiber word check with scratch printed
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05g_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
timeout -k 10 300 ./build/seal_batch_test 13 > $D/seal_batch.log 2>&1; echo "seal_batch rc=$?"; tail -1 $D/seal_batch.log
timeout -k 10 300 ./build/resnet_test $P $C fibercheck 8 2 4 > $D/fc.log 2>&1; echo "fc rc=$?"; grep "^batch" $D/fc.log
for v in "3 8 24" "4 8 32" "3 8 48" "4 6 24" "3 6 18" "2 8 16"; do
  set -- $v
  MHE_RESNET_FIBERS=$2 timeout -k 10 300 ./build/resnet_test $P $C $3 20 $1 > $D/t$1_f$2_i$3.log 2>&1
  rc=$?; echo "t$1 f$2 i$3 rc=$rc $(grep '^batch:' $D/t$1_f$2_i$3.log)" | tee -a $D/sweep.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
