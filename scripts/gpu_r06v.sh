# r06v: output primes per lift-pass workgroup (MHE_ICOL_PER 1 / 2 / 3 against the size rule): rescales and
# HMults at ResNet levels, ResNet-20 3 x 8
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06v_$(date +%H%M%S)
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
step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "rescale or hmult or moddown or rotate"
tail -1 $D/parity.log
for rep in 1 2; do
for per in 0 1 2 3; do
  for L in 25 17; do
    MHE_ICOL_PER=$per step u_${per}_${L}_$rep 300 python -u scripts/ubench_ops.py --limbs $L --ops rescale,rescale8,hmult,ks4 --reps 30
    grep '^{' $D/u_${per}_${L}_$rep.log | sed "s/}/, \"per\": $per}/" >> $D/ubench.jsonl
  done
done
done
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for per in 0 1 2; do
  MHE_ICOL_PER=$per LD_LIBRARY_PATH=fhe-gpt-2_amd MHE_RESNET_FIBERS=8 step resnet_$per 400 ./build/resnet_test $P $C 24 20 3
  echo "per=$per $(grep '^batch:' $D/resnet_$per.log)" | tee -a $D/resnet.txt
done
