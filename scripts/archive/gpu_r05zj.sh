# r05zj: the full GPU suite at the final round-5 HEAD (encoder FFT tail pass) + smoke
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05zj_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -rf > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a $D/rc.txt; tail -5 $D/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1; echo "smoke rc=$?" | tee -a $D/rc.txt
