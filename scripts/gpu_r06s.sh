# r06s: scalar first-phase twiddles in the ModDown / rescale / HMult-tail lift column passes (main) against
# build/vx/nocstw (HEAD before): parity subset, HMult bench 2 rounds, ResNet-level ops, ResNet-20 3 x 8.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06s_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $D/rc.txt
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 $D/$name.log; exit $rc; }
}
libpath() { if [ $1 = main ]; then echo $R/fhe-gpt-2_amd/libmhe.so; else echo $R/build/vx/$1/libmhe.so; fi; }
step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py
tail -1 $D/parity.log
for rep in 1 2; do
for lib in main nocstw; do
  MHE_LIB_PATH=$(libpath $lib) step bench_${lib}_$rep 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['modup_col_avg_launch_us'], d.get('valu_roofline',{}).get('frac'))" | tee -a $D/bench.txt
done
done
for lib in main nocstw; do
  MHE_LIB_PATH=$(libpath $lib) step u_${lib} 300 python -u scripts/ubench_ops.py --limbs 25 --ops rescale,rescale8,ks,ks4,hmult,ntt --reps 30
  grep '^{' $D/u_${lib}.log | sed "s/}/, \"v\": \"$lib\"}/" >> $D/ubench.jsonl
done
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for lib in main nocstw; do
  LD=$(dirname $(libpath $lib))
  LD_LIBRARY_PATH=$LD MHE_RESNET_FIBERS=8 step resnet_$lib 400 ./build/resnet_test $P $C 24 20 3
  echo "$lib $(grep '^batch:' $D/resnet_$lib.log)" | tee -a $D/resnet.txt
done
