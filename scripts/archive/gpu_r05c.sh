# r05c: the fault-injection batch test against this round's SEAL surface and round 4's (A/B: the
# round-4 library must fail the merged-rescale retry check), then counters at HEAD: rocprofv3 kernel
# trace of the HMult bench, PMC traffic passes, SQ counters of the two key-switch kernels
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05c_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
timeout -k 10 300 ./build/seal_batch_test 13 > $D/seal_batch_new.log 2>&1; echo "new rc=$?" | tee -a $D/rc.txt
grep -E "FAIL|nth|ALL PASSED|inject|retried|rescaled once|unchanged" $D/seal_batch_new.log
LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/build/var_old timeout -k 10 300 ./build/seal_batch_test 13 > $D/seal_batch_r04.log 2>&1; echo "r04 rc=$?" | tee -a $D/rc.txt
grep -E "FAIL|nth|ALL PASSED|rescaled once|unchanged" $D/seal_batch_r04.log
SKIP_TESTS=1 TAG=r05c bash scripts/gpu_round.sh > $D/round.log 2>&1; echo "round rc=$?" | tee -a $D/rc.txt
bash scripts/gpu_sq.sh > $D/sq.log 2>&1; echo "sq rc=$?" | tee -a $D/rc.txt
cat gpurun_out/pmc/traffic.log | tail -5
