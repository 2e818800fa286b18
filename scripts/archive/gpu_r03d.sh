# r03d: round evidence at HEAD -- pytest -m gpu, smoke, bench (default legs), rocprofv3 kernel-trace
# stats of the HMult leg, FETCH/WRITE traffic per HMult (8 per mhe_hmult_batch), and the SQ counter
# passes (VALU / LDS / waits) for the two key-switch kernels that bench.py's valu_roofline reads.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r03d bash scripts/gpu_round.sh || exit $?
rm -rf gpurun_out/pmc_sq1 gpurun_out/pmc_sq2
PMC_FILTER="k_ks_row_mac|k_modup_col" PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" bash scripts/gpu_pmc.sh || exit $?
mv gpurun_out/pmc/p1 gpurun_out/pmc_sq1
PMC_FILTER="k_ks_row_mac|k_modup_col" PMC_GROUPS="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" bash scripts/gpu_pmc.sh || exit $?
mv gpurun_out/pmc/p1 gpurun_out/pmc_sq2
mkdir -p gpurun_out/pmc_sq && cp -r gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 gpurun_out/pmc_sq/
python3 scripts/sq_json.py gpurun_out/pmc_sq 44 gpurun_out/r03d_sq_counters.json > /dev/null
find gpurun_out/pmc_sq gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 -name "*.csv" -delete
# one steady-state ResNet-20 image (2-image minus 1-image rocprofv3 run)
rm -rf gpurun_out/prof_rn1 gpurun_out/prof_rn2
bash scripts/gpu_prof_resnet_diff.sh || exit $?
python3 scripts/kstats.py diff gpurun_out/prof_rn1/rn_kernel_stats.csv gpurun_out/prof_rn2/rn_kernel_stats.csv > gpurun_out/r03d_resnet20_per_image_kernels.txt
