# r06x: ResNet-20 batch shapes at HEAD with the box's default 4 hardware queues: 3 x 8 against 4 x 8
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06x_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for shape in "24 3" "32 4" "24 3" "32 4"; do
  set -- $shape
  n=rn_${1}_${2}_$(date +%s)
  LD_LIBRARY_PATH=fhe-gpt-2_amd MHE_RESNET_FIBERS=8 timeout -k 10 400 ./build/resnet_test $P $C $1 20 $2 > $D/$n.log 2>&1
  rc=$?; echo "$n rc=$rc" >> $D/rc.txt; [ $rc -eq 0 ] || { tail -20 $D/$n.log; exit $rc; }
  echo "$1 images / $2 streams: $(grep '^batch:' $D/$n.log)" | tee -a $D/resnet.txt
done
