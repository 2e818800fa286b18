# r03zz: the whole GPU suite and smoke at the round's last HEAD (after the MIX ModUp occupancy change)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread > gpurun_out/r03zz_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zz_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r03zz_bench.log 2>&1 || exit $?
