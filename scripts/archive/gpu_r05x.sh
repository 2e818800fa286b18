# r05x: kernel composition of the seeded ResNet-20 3 x 8 batch (24 images) at HEAD
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05x_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
MHE_RESNET_FIBERS=8 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$D/p24 -o k --output-format csv -- $R/build/resnet_test $R/$P $R/$C 24 20 3 > $D/run24.log 2>&1
rc=$?; echo "rc=$rc $(grep '^batch:' $D/run24.log)"
find $D/p24 -name "*kernel_trace*" -delete
