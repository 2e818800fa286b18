# r05y: hoisted ModUp row pass through k_fwd_row3 (bit-reversed stores) -- parity subset (hoisted
# tests check every rotation word), elementwise / BSGS / rescale timings, ResNet-20 3 x 8
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05y_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py tests/test_seal_api.py
tail -1 $D/parity.log
grep -q " passed" $D/parity.log && ! grep -q "failed" $D/parity.log || exit 1
for NL in 25 31; do
  step u_L$NL 200 python -u scripts/ubench_ops.py --limbs $NL --ops add,mulplain,ntt,rescale8,bsgs --reps 40
  grep '^{' $D/u_L$NL.log
done
MHE_RESNET_FIBERS=8 step resnet 400 ./build/resnet_test $P $C 24 20 3
grep '^batch:' $D/resnet.log; tail -1 $D/resnet.log
