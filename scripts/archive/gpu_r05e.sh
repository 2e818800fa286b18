# r05e: ResNet-20 batch shape sweep (host threads x fibers) with hoisting on, then a rocprofv3 kernel
# summary of the default 8-image 2 x 4 batch
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05e_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "2 4 8" "2 6 12" "3 4 12" "4 2 8" "2 8 16" "4 4 16" "1 8 8" "3 3 9"; do
  set -- $v
  MHE_RESNET_FIBERS=$2 timeout -k 10 300 ./build/resnet_test $P $C $3 20 $1 > $D/t$1_f$2_i$3.log 2>&1
  rc=$?; echo "t$1 f$2 i$3 rc=$rc $(grep '^batch:' $D/t$1_f$2_i$3.log)" | tee -a $D/sweep.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
export TMPDIR=/tmp
MHE_RESNET_FIBERS=4 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o resnet8 --output-format csv -- $GRAFT_REPO_ROOT/build/resnet_test $GRAFT_REPO_ROOT/$P $GRAFT_REPO_ROOT/$C 8 20 2 > $D/prof.log 2>&1
echo "prof rc=$?" | tee -a $D/sweep.txt
find $D/prof -name "*kernel_trace*" -delete
