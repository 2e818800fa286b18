# r03zs: SQ counters of the two key-switch kernels at HEAD (after the ModUp twiddle staging)
# SQ counters of the two key-switch kernels in small groups (one rocprofv3 --pmc pass each, no
# trace domains), summarised per dispatch into gpurun_out/r03zf_sq_counters.json (scripts/sq_json.py)
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/sq"
rm -rf "$O"; mkdir -p "$O"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY" "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_ks_row_mac|k_modup_col" -d "$O/p$i" -o pmc --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 1 --warmup 1 --batch 8 --streams 1 --resnet-images 0 > "$O/p$i.log" 2>&1 || exit $?
done
python3 scripts/sq_json.py "$O" 44 gpurun_out/r03zf_sq_counters.json > gpurun_out/sq/sq.log 2>&1
find "$O" -name "*.csv" -delete
