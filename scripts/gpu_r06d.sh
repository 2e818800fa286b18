# r06d: the whole GPU suite (as the driver runs it) and smoke() at HEAD.
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06d_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -q -rf --durations=25 --timeout 700 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a $D/rc.txt
tail -30 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a $D/rc.txt; cat $D/smoke.log | tail -2
exit $rc
