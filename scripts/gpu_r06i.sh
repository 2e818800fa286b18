# r06i: seeded ResNet-20 batch, FP64 elementwise products (main) against build/vx/nowave (integer
# products): with the same seed the two libraries must print the same logit errors.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06i_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for lib in main nowave; do
  if [ $lib = main ]; then LD=$R/fhe-gpt-2_amd; else LD=$R/build/vx/$lib; fi
  LD_LIBRARY_PATH=$LD MHE_RESNET_SEED=7 MHE_RESNET_FIBERS=8 timeout -k 10 300 ./build/resnet_test $P $C 8 20 1 > $D/resnet_$lib.log 2>&1
  rc=$?; echo "resnet_$lib rc=$rc" | tee -a $D/rc.txt; [ $rc -eq 0 ] || exit $rc
  grep 'logit error' $D/resnet_$lib.log > $D/err_$lib.txt
done
if cmp -s $D/err_main.txt $D/err_nowave.txt; then echo "seeded logit errors identical"; else echo "seeded logit errors DIFFER"; diff $D/err_main.txt $D/err_nowave.txt | head -20; fi
