# r05k: lazy FP butterflies in the generic passes, prime-major row passes, k_icol_lift with the
# FP lift and LDS twiddles -- parity, op micro-timings, HMult bench, ResNet-20 3 x 8 batch
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05k_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt; tail -4 $D/$name.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py
for L in 25 31; do
  step ubench_L$L 300 python -u scripts/ubench_ops.py --limbs $L --ops rescale,rescale8,ks,ks4s,ntt --reps 40
  grep '^{' $D/ubench_L$L.log
done
step bench_hmult 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
grep '^{' $D/bench_hmult.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"
MHE_RESNET_FIBERS=8 step resnet_3x8 400 ./build/resnet_test $P $C 24 20 3
