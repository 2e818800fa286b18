set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/sweep.log
for s in ${STREAMS:-3 4 6}; do
  echo "== streams=$s" >> gpurun_out/sweep.log
  timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 2 --streams $s >> gpurun_out/sweep.log 2>&1 || exit $?
done
