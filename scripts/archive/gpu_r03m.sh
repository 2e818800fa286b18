# r03m: conflict-free LDS image in the row passes (MHE_ROW_SWZ) + row epilogue prefetch: parity,
# per-op A/B vs HEAD (build/var/base) and the build without the swizzle (build/var/noswz), LDS
# conflict counters of rescale / NTT, ResNet-20 4 images with lockstep 0 / 2.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || exit $?
for lib in base noswz cur base noswz cur; do
  if [ $lib = cur ]; then unset MHE_LIB_PATH; else export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"; fi
  timeout -k 10 200 python scripts/ubench_ops.py >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
done
unset MHE_LIB_PATH
for op in rescale ntt; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$PWD/$O/pmc_$op" -o pmc --output-format csv -- python3 scripts/ubench_ops.py --ops $op --reps 4 > $O/pmc_$op.log 2>&1 || exit $?
  python3 scripts/pmc_summary.py $O/pmc_$op > $O/pmc_$op.txt 2>&1
done
find $O -name '*.csv' -delete
for v in 0 2 0 2; do
  MHE_RESNET_LOCKSTEP=$v MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 400 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 4 20 4 > $O/resnet_ls${v}_$(date +%s).log 2>&1 || exit $?
done
