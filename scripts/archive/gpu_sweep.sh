# parity tests, then a bench sweep over an env knob (SWEEP_VAR over SWEEP_VALUES)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/sweep.log
for v in $SWEEP_VALUES; do
  echo "== $SWEEP_VAR=$v" >> gpurun_out/sweep.log
  env $SWEEP_VAR=$v timeout -k 10 300 python bench.py --no-cpu --steps 6 --warmup 2 ${BENCH_ARGS:-} >> gpurun_out/sweep.log 2>&1 || exit $?
done
