# rocprofv3 kernel stats of boot_test (logn 14, 4 bootstraps) -> gpurun_out/prof_boot
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_boot
timeout -k 10 300 ./build/boot_test 14 4 > gpurun_out/prof_boot/plain.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_boot" -o boot --output-format csv -- "$R/build/boot_test" 14 4 > gpurun_out/prof_boot/boot.log 2>&1
rc=$?
find gpurun_out/prof_boot -name "*kernel_trace*" -delete
exit $rc
