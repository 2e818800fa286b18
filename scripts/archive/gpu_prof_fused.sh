set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export MHE_KS_FUSED=${MHE_KS_FUSED:-1}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/pmc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o fused --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1 || exit $?
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_ks_row_mac|k_fwd_col" -d "$R/gpurun_out/pmc/p$i" -o pmc --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 1 --warmup 0 --batch 2 > "gpurun_out/pmc/p$i.log" 2>&1 || exit $?
done
