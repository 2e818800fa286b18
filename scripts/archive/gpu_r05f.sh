# r05f: rescale / key-switch micro-timings at ResNet levels with kernel trace + counters of the
# rescale launch sequence, and a wider ResNet-20 batch-shape sweep
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05f_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
for L in 25 31; do
  timeout -k 10 300 python -u scripts/ubench_ops.py --limbs $L --ops rescale,rescale4,rescale8,ks,ks4,ks4s,ntt --reps 40 > $D/ubench_L$L.log 2>&1
  echo "ubench L$L rc=$?"; grep '^{' $D/ubench_L$L.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/prof -o resc --output-format csv -- python3 $R/scripts/ubench_ops.py --limbs 25 --ops rescale8 --reps 20 > $D/prof.log 2>&1
echo "prof rc=$?"
find $D/prof -name "*kernel_trace*" -delete
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "Rescale|LastInv" -d $R/$D/pmc$i -o pmc --output-format csv -- python3 $R/scripts/ubench_ops.py --limbs 25 --ops rescale8 --reps 5 > $D/pmc$i.log 2>&1
  echo "pmc$i rc=$?"
done
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "2 8 16" "3 8 24" "2 16 32" "1 16 16"; do
  set -- $v
  MHE_RESNET_FIBERS=$2 timeout -k 10 300 ./build/resnet_test $P $C $3 20 $1 > $D/t$1_f$2_i$3.log 2>&1
  rc=$?; echo "t$1 f$2 i$3 rc=$rc $(grep '^batch:' $D/t$1_f$2_i$3.log)" | tee -a $D/sweep.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
