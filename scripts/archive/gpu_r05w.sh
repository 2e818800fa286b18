# r05w: the default bench line at HEAD (seeded ResNet runner), and the seeded ResNet-20 3 x 8 batch
# twice: the per-image logit errors must repeat
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05w_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
timeout -k 10 900 python -u bench.py > $D/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' $D/bench.log > $D/bench.json; [ $rc -eq 0 ] || exit $rc
for r in a b; do
  MHE_RESNET_FIBERS=8 timeout -k 10 400 ./build/resnet_test $P $C 24 20 3 > $D/resnet_$r.log 2>&1; rc=$?
  echo "$r rc=$rc $(grep '^batch:' $D/resnet_$r.log) $(grep 'batch image' $D/resnet_$r.log | awk '{printf "%s ", $7}')" | tee -a $D/summary.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
