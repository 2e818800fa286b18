# r04m: PMC passes on the hoisted key MAC (8 inputs x 7 rotations, 31 limbs, one call): HBM fetch,
# L2 hits / misses, SQ instruction / wait counters -- one rocprofv3 run per counter group
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/r04m"
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "hoist|k_ks_row_mac|k_fwd_row" -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$R/scripts/ubench_ops.py" --ops bsgs --bsgs 8x7 --limbs 31 --reps 1 > "$OUT/p$i.log" 2>&1 || exit $?
done
