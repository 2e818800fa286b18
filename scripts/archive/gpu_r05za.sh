# r05za: forward column pass with the first post-barrier twiddles loaded with the data -- parity, then A/B against
# build/vx/base (HEAD before the change) on op timings, the HMult bench and ResNet-20 3 x 8 (libmhe_seal loads
# libmhe.so through its rpath, so the ResNet A/B swaps LD_LIBRARY_PATH in front of it)
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05za_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py tests/test_seal_api.py
tail -2 $D/parity.log
grep -q " passed" $D/parity.log && ! grep -q "failed" $D/parity.log || exit 1
for lib in main base; do
  if [ $lib = main ]; then L=$GRAFT_REPO_ROOT/fhe-gpt-2_amd/libmhe.so; LD=$GRAFT_REPO_ROOT/fhe-gpt-2_amd; else L=$GRAFT_REPO_ROOT/build/vx/$lib/libmhe.so; LD=$GRAFT_REPO_ROOT/build/vx/$lib; fi
  for NL in 25 31; do
    MHE_LIB_PATH=$L step u_${lib}_L$NL 200 python -u scripts/ubench_ops.py --limbs $NL --ops rescale8,ks4s,ks,ntt,mulplain --reps 40
    grep '^{' $D/u_${lib}_L$NL.log | sed "s/}/, \"v\": \"$lib\"}/" >> $D/all.jsonl
  done
  MHE_LIB_PATH=$L step bench_$lib 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'])" | tee -a $D/bench.txt
  LD_LIBRARY_PATH=$LD MHE_RESNET_FIBERS=8 step resnet_$lib 400 ./build/resnet_test $P $C 24 20 3
  echo "$lib $(grep '^batch:' $D/resnet_$lib.log) $(tail -1 $D/resnet_$lib.log)" | tee -a $D/resnet.txt
done
