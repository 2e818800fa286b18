# parity tests -> smoke -> bench -> rocprofv3 kernel-trace summary; stop at the first GPU failure
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -x --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
[ -n "${NO_PROF:-}" ] && exit 0
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1 || exit $?
