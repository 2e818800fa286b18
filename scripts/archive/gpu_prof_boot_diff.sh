# Per-bootstrap kernel stats (logn 14): rocprofv3 stats of boot_test with 2 and 6 bootstraps; the
# difference is 4 steady-state bootstraps (scripts/kstats.py diff).
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for k in 2 6; do
  mkdir -p gpurun_out/prof_boot$k
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_boot$k" -o boot --output-format csv -- "$R/build/boot_test" 14 $k > gpurun_out/prof_boot$k/boot.log 2>&1
  rc=$?
  find gpurun_out/prof_boot$k -name "*kernel_trace*" -delete
  [ $rc -eq 0 ] || exit $rc
done
