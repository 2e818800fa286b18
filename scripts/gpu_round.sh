# Round evidence: parity tests -> smoke -> bench -> rocprofv3 kernel-trace stats -> PMC traffic passes.
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG="${TAG:-run}"
mkdir -p gpurun_out/prof gpurun_out/pmc
rc=0
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
fi
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o $TAG --output-format csv -- python3 "$R/bench.py" --no-cpu --resnet-images 0 --streams 1 --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_trace*" -delete
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "^(k_|void k_)" -d "$R/gpurun_out/pmc/$c" -o pmc --output-format csv -- python3 "$R/bench.py" --no-cpu --resnet-images 0 --streams 1 --steps 1 --warmup 0 --batch 8 > "gpurun_out/pmc/$c.log" 2>&1 || exit $?
done
# 8 HMults in the run (one mhe_hmult_batch call, the bench's default launch shape)
python3 scripts/traffic.py gpurun_out/pmc 8 gpurun_out/pmc/traffic.json > gpurun_out/pmc/traffic.log 2>&1
find gpurun_out/pmc -name "*.csv" -delete
exit $rc
