# r03u: row-pass epilogue prefetch selected by launch size (MHE_ROW_PRE_MAX_WG: 0 never, 8192
# default, 1e9 always): parity file, C2 HMult leg and per-op timings at ResNet levels, same box.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || exit $?
for v in 0 8192 1000000000 0 8192 1000000000; do
  MHE_ROW_PRE_MAX_WG=$v timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > $O/hm_${v}_$(date +%s).json 2>> $O/err.log || exit $?
  MHE_ROW_PRE_MAX_WG=$v timeout -k 10 200 python scripts/ubench_ops.py --ops rescale,rescale4,ks,ks4,hmult >> $O/ops_$v.jsonl 2>> $O/err.log || exit $?
done
