# r03zf: round evidence at HEAD after the ModUp twiddle staging -- the whole GPU suite, smoke, the default bench line,
# rocprofv3 kernel-trace stats + PMC traffic of the HMult leg (scripts/gpu_round.sh), and one
# steady-state ResNet-20 image's kernels and launches (2-image minus 1-image rocprofv3 runs).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r03zf bash scripts/gpu_round.sh || exit $?
rm -rf gpurun_out/prof_rn1 gpurun_out/prof_rn2
bash scripts/gpu_prof_resnet_diff.sh || exit $?
python3 scripts/kstats.py diff gpurun_out/prof_rn1/rn_kernel_stats.csv gpurun_out/prof_rn2/rn_kernel_stats.csv > gpurun_out/r03zf_resnet20_per_image_kernels.txt
timeout -k 10 400 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > gpurun_out/r03zf_resnet20_4images.log 2>&1 || exit $?
# ModUp output-prime groups per digit with the LDS twiddles (<= 5 primes per group stay in LDS)
for g in 9 12 7 9 12 7; do
  MHE_KS_COLGROUPS=$g timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > gpurun_out/r03zf_colgroups_${g}_$(date +%s).json 2>> gpurun_out/r03zf_err.log || exit $?
done
