# tests (new: key export/import, cnn CLI), bench with the in-process ResNet leg, and resnet_test
# under rocprofv3 kernel-trace (1 stream, then 4) to locate the host fault seen under the profiler.
# Kernel-trace CSVs are dropped (the stats CSVs stay) so gpurun_out stays under 64 MiB.
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_resnet
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --durations=10 --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
export TMPDIR=/tmp
for cfg in "r1 1 1" "r4 4 4"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_resnet" -o $1 --output-format csv -- "$R/build/resnet_test" "$R/tests/golden/resnet/resnet20_params.bin" "$R/tests/golden/comp" $2 20 $3 > gpurun_out/prof_resnet/$1.log 2>&1
  echo "rc=$?" >> gpurun_out/prof_resnet/$1.log
  rm -f gpurun_out/prof_resnet/*kernel_trace.csv
done
exit $rc
