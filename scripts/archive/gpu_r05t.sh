# r05t: kernel stats at HEAD (HMult bench on one stream, rescale / key-switch ops at 25 limbs) and an
# A/B of the row passes' up-front epilogue prefetch threshold (MHE_ROW_PRE_MAX: 8192 workgroups
# vs 0 = grouped loads everywhere) on ops, HMult and ResNet-20 3 x 8
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05t_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$D/hm -o hm --output-format csv -- python3 $R/bench.py --no-cpu --streams 1 --steps 3 --warmup 1 --resnet-images 0 > $D/hm.log 2>&1 || exit $?
find $D/hm -name "*kernel_trace*" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/ops -o ops --output-format csv -- python3 $R/scripts/ubench_ops.py --limbs 25 --ops rescale8,ks4s --reps 20 > $D/ops.log 2>&1 || exit $?
find $D/ops -name "*kernel_trace*" -delete
for pm in 8192 0; do
  for NL in 25 31; do
    MHE_ROW_PRE_MAX=$pm timeout -k 10 200 python -u scripts/ubench_ops.py --limbs $NL --ops rescale8,rescale,ks4s,ks --reps 40 > $D/u_${pm}_$NL.log 2>&1 || exit $?
    grep '^{' $D/u_${pm}_$NL.log | sed "s/}/, \"pre_max\": $pm}/" >> $D/all.jsonl
  done
  MHE_ROW_PRE_MAX=$pm MHE_RESNET_FIBERS=8 timeout -k 10 400 ./build/resnet_test $P $C 24 20 3 > $D/resnet_$pm.log 2>&1; rc=$?
  echo "pre_max $pm rc=$rc $(grep '^batch:' $D/resnet_$pm.log)" | tee -a $D/summary.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
