# r05a: hoisted-rotation tests that really hoist (mhe_ctx_set_hoist + check), the FiberBatch
# shape test, and the ResNet-20 fiber-batch vs alone word check (hoisting off / on)
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05a_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py \
  > $D/pytest_batch.log 2>&1
rc=$?; echo "pytest_batch rc=$rc" | tee -a $D/rc.txt; tail -3 $D/pytest_batch.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 ./build/resnet_test $P $C fibercheck 4 2 2 > $D/fc_4_2_2.log 2>&1
rc=$?; echo "fc_4_2_2 rc=$rc" | tee -a $D/rc.txt; tail -4 $D/fc_4_2_2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 ./build/resnet_test $P $C fibercheck 8 2 4 > $D/fc_8_2_4_a.log 2>&1
rc=$?; echo "fc_8_2_4_a rc=$rc" | tee -a $D/rc.txt; tail -4 $D/fc_8_2_4_a.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 ./build/resnet_test $P $C fibercheck 8 2 4 > $D/fc_8_2_4_b.log 2>&1
rc=$?; echo "fc_8_2_4_b rc=$rc" | tee -a $D/rc.txt; tail -4 $D/fc_8_2_4_b.log
