# PMC passes over a short HMult run (separate rocprofv3 invocation per counter group, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes: no --pmc together with trace domains)
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu --steps 1 --warmup 1 --batch 8 --streams 1 --resnet-images 0"
FILTER="${PMC_FILTER:-k_ks_row_mac|k_fwd_col|k_fwd_row}"
i=0
for grp in ${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$FILTER" -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || exit $?
done
