# r06c: the fused key MAC with its keys and accumulators in the row transform's last layout (no
# transpose back per digit, MHE_KS_FL) against build/vx/nofl (the r06b kernel) and build/vx/flocc2
# (FL at 2 waves/SIMD): parity first, then same-box HMult bench A/B and ResNet-level ops.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06c_$(date +%H%M%S)
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
for rep in 1 2; do
for lib in main nofl flocc2; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  MHE_LIB_PATH=$L step bench_${lib}_$rep 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['modup_col_avg_launch_us'], d.get('valu_roofline',{}).get('frac'))" | tee -a $D/bench.txt
done
done
for lib in main nofl flocc2; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  MHE_LIB_PATH=$L step u_${lib} 300 python -u scripts/ubench_ops.py --limbs 25 --ops ks,ks4,ks4s,rot4,hmult,bsgs --reps 30
  grep '^{' $D/u_${lib}.log | sed "s/}/, \"v\": \"$lib\"}/" >> $D/ubench.jsonl
done
step prof 400 rocprofv3 --kernel-trace --stats -d $R/$D/hm -o hm --output-format csv -- python3 $R/bench.py --no-cpu --streams 1 --steps 3 --warmup 1 --resnet-images 0
find $D/hm -name "*kernel_trace*" -delete
# the 48-image ResNet-20 batch (3 threads x 8 fibers, two batches per thread)
# under rocprofv3's kernel trace, once, with guard-paged fiber stacks and the fault handler that
# names the faulting address (tests/cpp/resnet_test.cpp on_fault)
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
MHE_RESNET_FIBERS=8 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$D/p48 -o k --output-format csv -- $R/build/resnet_test $R/$P $R/$C 48 20 3 > $D/run48.log 2>&1
rc=$?; echo "run48 rc=$rc $(grep '^batch:' $D/run48.log)" | tee -a $D/rc.txt
find $D/p48 -name "*kernel_trace*" -delete
exit $rc
