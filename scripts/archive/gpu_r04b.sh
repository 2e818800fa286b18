# r04b: GPT-2 block pieces (GELU vs poly.py, reference and indicator variants) and the block at GPT-2 width
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpt2.py -m gpu -x -v -s --timeout 800 --timeout-method thread -k "block" > gpurun_out/r04b_gpt2.log 2>&1 || exit $?
