# r05r: k_col_lift2 for the HMult tail column pass + row-pass twiddle prefetch: parity subset,
# ResNet-20 3 x 8, HMult bench (twice)
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05r_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt; tail -2 $D/$name.log
  [ $rc -eq 0 ] || exit $rc
}
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py tests/test_seal_api.py
MHE_RESNET_FIBERS=8 step resnet_3x8 400 ./build/resnet_test $P $C 24 20 3
step bench_hmult 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
step bench_hmult2 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
