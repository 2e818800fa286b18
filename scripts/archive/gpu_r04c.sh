# r04c: bootstrap trace parity (new boot mode), the conv/BN/ReLU trace, bootstrapping end to end with
# the reference-order LT diagonals, ResNet logits
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_trace_parity.py tests/test_seal_api.py -m gpu -x -v -s --timeout 800 --timeout-method thread > gpurun_out/r04c_trace.log 2>&1 || exit $?
