# r03d: bootstrapping / ResNet accuracy with the Remez-generated EvalMod cosine, then the round
# evidence at HEAD (pytest -m gpu, smoke, bench, kernel-trace stats, FETCH/WRITE traffic) and the
# SQ counter passes bench.py's valu_roofline reads.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for ln in 14 13 12; do timeout -k 10 300 ./build/boot_test $ln 2 > gpurun_out/r03d_boot$ln.log 2>&1 || exit $?; done
timeout -k 10 600 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > gpurun_out/r03d_resnet.log 2>&1 || exit $?
TAG=r03d bash scripts/gpu_round.sh || exit $?
PMC_FILTER="k_ks_row_mac|k_modup_col" PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" bash scripts/gpu_pmc.sh || exit $?
python3 scripts/sq_json.py gpurun_out/pmc 44 gpurun_out/r03d_sq_counters.json > /dev/null
find gpurun_out/pmc -name "*.csv" -delete
