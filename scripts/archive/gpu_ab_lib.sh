# Same-box A/B of two libmhe builds on the HMult leg: ab/libmhe_base.so vs the tree's libmhe.so,
# alternating, after a parity subset on the tree's library
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "hmult or switch_key or variants or prepared" > gpurun_out/ab/pytest.log 2>&1 || exit $?
B="timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 20"
for i in 1 2 3; do
  MHE_LIB_PATH=$GRAFT_REPO_ROOT/ab/libmhe_base.so $B > gpurun_out/ab/base_$i.json 2>/dev/null || exit $?
  $B > gpurun_out/ab/new_$i.json 2>/dev/null || exit $?
done
for f in gpurun_out/ab/*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"avg_launch_us": [0-9.]*' $f) $(grep -o '"modup_col_avg_launch_us": [0-9.]*' $f)"; done > gpurun_out/ab/summary.txt
