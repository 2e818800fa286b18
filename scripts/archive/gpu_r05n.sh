# r05n: per-image kernel composition of the ResNet-20 3 x 8 batch, free of setup: kernel stats of
# a 24-image and a 48-image run, differenced (scripts/kstats.py diff)
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05n_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for N in 24 48; do
  MHE_RESNET_FIBERS=8 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$D/p$N -o k --output-format csv -- $R/build/resnet_test $R/$P $R/$C $N 20 3 > $D/run$N.log 2>&1
  rc=$?; echo "n$N rc=$rc $(grep '^batch:' $D/run$N.log)"
  find $D/p$N -name "*kernel_trace*" -delete
  [ $rc -eq 0 ] || exit $rc
done
