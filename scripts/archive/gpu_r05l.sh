# r05l: k_icol_lift (FP lift, LDS twiddles, lazy sweep) + prime-major row passes: parity and
# rescale / key-switch timings with kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05l_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt; tail -3 $D/$name.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py
for L in 25 31; do
  step ubench_L$L 300 python -u scripts/ubench_ops.py --limbs $L --ops rescale,rescale8,ks,ks4s,ntt --reps 40
  grep '^{' $D/ubench_L$L.log | sort -u
done
step prof 300 rocprofv3 --kernel-trace --stats -d $R/$D/prof -o ops --output-format csv -- python3 $R/scripts/ubench_ops.py --limbs 25 --ops rescale8,ks4s --reps 20
find $D/prof -name "*kernel_trace*" -delete
