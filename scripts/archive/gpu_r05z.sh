# r05z(b): GPU busy fraction and idle gaps of the ResNet-20 3 x 8 batch: kernel trace of a 24-image run, reduced on
# the box to the union of kernel intervals over the batch window (scripts/busy.py)
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05z_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
MHE_RESNET_FIBERS=8 timeout -k 10 500 rocprofv3 --kernel-trace -d $R/$D/t -o k --output-format csv -- $R/build/resnet_test $R/$P $R/$C 24 20 3 > $D/run.log 2>&1
rc=$?; echo "rc=$rc $(grep '^batch:' $D/run.log)"
[ $rc -eq 0 ] || exit $rc
python3 scripts/busy.py $(find $D/t -name "*kernel_trace.csv") > $D/busy.txt; cat $D/busy.txt
find $D/t -name "*kernel_trace*" -delete
