# r05o: ResNet-20 3 x 8 throughput at HEAD (k_icol_lift FP lift / LDS twiddles), twice, and a
# 48-image run (two batches per thread) without the profiler
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05o_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "24 a" "24 b" "48 c"; do
  set -- $v
  MHE_RESNET_FIBERS=8 timeout -k 10 400 ./build/resnet_test $P $C $1 20 3 > $D/run_$2.log 2>&1
  rc=$?; echo "n$1 $2 rc=$rc $(grep '^batch:' $D/run_$2.log)" | tee -a $D/summary.txt
  [ $rc -eq 0 ] || exit $rc
done
