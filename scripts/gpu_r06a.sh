# r06a: fused key MAC with the input limb peeled out of the digit loop, buffer loads of the packed
# ModUp digits and the prepared key as doubles, at 3 waves/SIMD.  Parity of the key-switch paths
# first, then same-box A/B of the HMult bench and ResNet-level ops against build/vx/occ2 (same code
# at 2 waves/SIMD) and build/vx/head (round-5 HEAD), then a rocprofv3 kernel trace of the new HMult.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06a_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/rc.txt
  [ $rc -eq 0 ] || exit $rc
}
step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py
tail -2 $D/parity.log
step resnet3 600 ./build/resnet_test tests/golden/resnet/resnet20_params.bin tests/golden/comp 3
grep -E "max \|logit error\| vs|setup" $D/resnet3.log
for rep in 1 2; do
for lib in main occ2 head; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  MHE_LIB_PATH=$L step bench_${lib}_$rep 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['achieved'], d.get('valu_roofline',{}).get('frac'))" | tee -a $D/bench.txt
done
done
for lib in main head; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  for NL in 25 31; do
    MHE_LIB_PATH=$L step u_${lib}_L$NL 200 python -u scripts/ubench_ops.py --limbs $NL --ops ks,ks4,ks4s,rot4,hmult --reps 30
    grep '^{' $D/u_${lib}_L$NL.log | sed "s/}/, \"v\": \"$lib\"}/" >> $D/ubench.jsonl
  done
done
step prof 400 rocprofv3 --kernel-trace --stats -d $R/$D/hm -o hm --output-format csv -- python3 $R/bench.py --no-cpu --streams 1 --steps 3 --warmup 1 --resnet-images 0
find $D/hm -name "*kernel_trace*" -delete
