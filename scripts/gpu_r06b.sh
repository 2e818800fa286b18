# r06b: key-format and occupancy variants of the fused key MAC.  Parity of the key-switch paths
# (both prepared formats, mixed in one launch) and the fault-injection driver first; then same-box
# A/B of the HMult bench over main (3 waves/SIMD), build/vx/occ2 and build/vx/occ2kpf (2 waves,
# keys one digit ahead); ResNet-level ops with the doubles (MHE_KEY_FMT=1) and 48-bit (=2) key
# formats; the ResNet-20 leg of bench.py with either format.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06b_$(date +%H%M%S)
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
for lib in main occ2 occ2kpf; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  MHE_LIB_PATH=$L step bench_${lib}_$rep 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['modup_col_avg_launch_us'], d.get('valu_roofline',{}).get('frac'))" | tee -a $D/bench.txt
done
done
for lib in main occ2 occ2kpf; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  for F in 1 2; do
    MHE_KEY_FMT=$F MHE_LIB_PATH=$L step u_${lib}_f$F 300 python -u scripts/ubench_ops.py --limbs 25 --ops ks,ks4,ks4s,rot4,hmult --reps 30
    grep '^{' $D/u_${lib}_f$F.log | sed "s/}/, \"v\": \"$lib\", \"fmt\": $F}/" >> $D/ubench.jsonl
  done
done
for F in 1 2; do
  MHE_KEY_FMT=$F step resnet_f$F 500 python -u bench.py --no-cpu --steps 3 --warmup 1 --resnet-key-draws 0
  grep '^{' $D/resnet_f$F.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['resnet20']; print('fmt $F', r['sec_per_image_1stream'], r['images_per_s'], r['bootstrap_s_per_image'], r['logit_check']['max_abs_err_per_image']['vs_approx_relu'][:4], r['fallbacks'])" | tee -a $D/resnet.txt
done
