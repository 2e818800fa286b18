# r05b: hoisting on by default -- batch parity, the fault-injection batch test, fiber-batch word check,
# the ResNet-shape bootstrap trace replay, then the bench line
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05b_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt; tail -4 $D/$name.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
step seal_batch 300 ./build/seal_batch_test 13
step pytest_batch 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py
step fc_8_2_4 300 ./build/resnet_test $P $C fibercheck 8 2 4
step boot_trace16 900 python -u -m pytest -x -v -s --timeout 850 --timeout-method thread -m gpu "tests/test_trace_parity.py::test_sparse_bootstrap_resnet_shape_matches_oracle"
step bench 600 python -u bench.py
