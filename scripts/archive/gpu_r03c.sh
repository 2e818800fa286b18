# r03c: caller-sequence trace parity vs the oracle, then the full bench line
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_trace_parity.py -x -v -s --timeout 800 --timeout-method thread > gpurun_out/r03c_trace.log 2>&1
rc=$?
timeout -k 10 600 python bench.py > gpurun_out/r03c_bench.log 2>&1 || exit $?
exit $rc
