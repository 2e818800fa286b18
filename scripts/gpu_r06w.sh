# r06w: output primes per lift-pass workgroup at batched sizes, MHE_ICOL_G 3 (main) / 4 / 5 (builds
# build/vx/icolg4, icolg5): parity, rescales and HMults at ResNet levels, HMult bench, ResNet-20 3 x 8
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06w_$(date +%H%M%S)
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
for lib in icolg4 icolg5; do
  MHE_LIB_PATH=$(libpath $lib) step parity_$lib 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py
  echo "$lib $(tail -1 $D/parity_$lib.log)"
done
for rep in 1 2; do
for lib in main icolg4 icolg5; do
  for L in 25 17; do
    MHE_LIB_PATH=$(libpath $lib) step u_${lib}_${L}_$rep 300 python -u scripts/ubench_ops.py --limbs $L --ops rescale,rescale8,hmult --reps 30
    grep '^{' $D/u_${lib}_${L}_$rep.log | sed "s/}/, \"v\": \"$lib\"}/" >> $D/ubench.jsonl
  done
done
done
for lib in main icolg4 icolg5; do
  MHE_LIB_PATH=$(libpath $lib) step bench_${lib} 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['modup_col_avg_launch_us'])" | tee -a $D/bench.txt
done
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for lib in main icolg4 icolg5; do
  LD=$(dirname $(libpath $lib))
  LD_LIBRARY_PATH=$LD MHE_RESNET_FIBERS=8 step resnet_$lib 400 ./build/resnet_test $P $C 24 20 3
  echo "$lib $(grep '^batch:' $D/resnet_$lib.log)" | tee -a $D/resnet.txt
done
