# r05q: A/B of the row-pass twiddle prefetch (main: MHE_ROW_TWPF=1, build/vx/pf0: 0) -- parity of
# the main build, op micro-timings and the HMult bench for both, ResNet-20 3 x 8 for both
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05q_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt
  [ $rc -eq 0 ] || exit $rc
}
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py
for rep in 1 2; do
for lib in main pf0; do
  if [ $lib = main ]; then L=$GRAFT_REPO_ROOT/fhe-gpt-2_amd/libmhe.so; else L=$GRAFT_REPO_ROOT/build/vx/$lib/libmhe.so; fi
  for NL in 25 31; do
    MHE_LIB_PATH=$L step u_${lib}_L${NL}_$rep 200 python -u scripts/ubench_ops.py --limbs $NL --ops rescale8,ks4s,ntt,rescale --reps 40
    grep '^{' $D/u_${lib}_L${NL}_$rep.log | sed "s/}/, \"v\": \"$lib\"}/" >> $D/all.jsonl
  done
  MHE_LIB_PATH=$L step bench_${lib}_$rep 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'])" | tee -a $D/bench.txt
done
done
