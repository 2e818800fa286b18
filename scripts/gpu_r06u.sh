# r06u (round-6 end, final HEAD): the default bench line at HEAD, the rocprofv3 kernel trace of the HMult bench on one stream
# (the roofline's per-launch durations), PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and
# the SQ counters of the two key-switch kernels, every counter pass its own rocprofv3 run.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06u_$(date +%H%M%S)
mkdir -p $D/pmc $D/sq
echo "logs in $D"
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > $D/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' $D/bench.log > $D/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$D/hm -o hm --output-format csv -- python3 $R/bench.py --no-cpu --streams 1 --steps 3 --warmup 1 --resnet-images 0 > $D/hm.log 2>&1 || exit $?
find $D/hm -name "*kernel_trace*" -delete
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "^(k_|void k_)" -d $R/$D/pmc/$c -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --resnet-images 0 --streams 1 --steps 1 --warmup 0 --batch 8 > $D/pmc/$c.log 2>&1 || exit $?
done
python3 scripts/traffic.py $D/pmc 8 $D/traffic.json > $D/pmc/traffic.log 2>&1
find $D/pmc -name "*.csv" -delete
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY" "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_ks_row_mac|k_modup_col" -d $R/$D/sq/p$i -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 1 --batch 8 --streams 1 --resnet-images 0 > $D/sq/p$i.log 2>&1 || exit $?
done
python3 scripts/sq_json.py $D/sq 44 $D/sq_counters.json > $D/sq/sq.log 2>&1
find $D/sq -name "*.csv" -delete
