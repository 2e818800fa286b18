# bench sweep over env settings: SWEEP="A=1 B=2;A=3 B=4" (parity tests first unless NOTEST=1)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/sweep.log
IFS=';'
for cfg in $SWEEP; do
  echo "== $cfg" >> gpurun_out/sweep.log
  IFS=' ' 
  env $cfg timeout -k 10 300 python bench.py --no-cpu --steps 6 --warmup 2 ${BENCH_ARGS:-} >> gpurun_out/sweep.log 2>&1 || exit $?
  IFS=';'
done
