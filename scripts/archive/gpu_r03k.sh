# r03k: generic NTT passes with twiddles loaded up front (build/var/twp): parity with it, per-op A/B
# at ResNet levels, per-op kernel breakdown, key-switch chunk / column-group sweep at L = 31, SQ + HBM
# counters of one L = 31 key switch.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
MHE_LIB_PATH=$PWD/build/var/twp/libmhe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity_twp.log 2>&1 || exit $?
for lib in cur twp cur twp; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 python scripts/ubench_ops.py >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
done
export MHE_LIB_PATH="$PWD/build/var/twp/libmhe.so"
for op in ks rescale ntt; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_$op" -o p --output-format csv -- python3 scripts/ubench_ops.py --ops $op --reps 20 > /dev/null 2>> $O/ops.err || exit $?
  python3 scripts/kstats.py $(find $O/prof_$op -name 'p_kernel_stats.csv' | head -1) > $O/k_twp_$op.txt || exit $?
done
for fc in 4 8 16; do
  MHE_KS_FCHUNK=$fc timeout -k 10 200 python scripts/ubench_ops.py --ops ks,rot4 --reps 30 | sed "s/}/, \"fchunk\": $fc}/" >> $O/sweep.jsonl 2>> $O/ops.err || exit $?
done
for cg in 4 16; do
  MHE_KS_COLGROUPS=$cg timeout -k 10 200 python scripts/ubench_ops.py --ops ks,rot4 --reps 30 | sed "s/}/, \"colgroups\": $cg}/" >> $O/sweep.jsonl 2>> $O/ops.err || exit $?
done
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$PWD/$O/pmc$i" -o pmc --output-format csv -- python3 scripts/ubench_ops.py --ops ks --reps 4 > $O/pmc$i.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py $O > $O/pmc_summary.txt 2>&1
find $O -name '*.csv' ! -name 'p_kernel_stats.csv' -delete
exit 0
