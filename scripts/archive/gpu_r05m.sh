# r05m: A/B of the row-pass launch order (MHE_ROW_PM) and the prefetching row pass's occupancy
# (build/vx/occ1: no 3-wave bound) on rescale / key-switch micro-timings and the HMult bench
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05m_$(date +%H%M%S)
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
for lib in main occ1; do
  if [ $lib = main ]; then export MHE_LIB_PATH=$GRAFT_REPO_ROOT/fhe-gpt-2_amd/libmhe.so; else export MHE_LIB_PATH=$GRAFT_REPO_ROOT/build/vx/$lib/libmhe.so; fi
  for pm in 1 0; do
    for L in 25 31; do
      MHE_ROW_PM=$pm step u_${lib}_pm${pm}_L$L 200 python -u scripts/ubench_ops.py --limbs $L --ops rescale8,ks4s,ntt --reps 40
      grep '^{' $D/u_${lib}_pm${pm}_L$L.log | sed "s/}/, \"pm\": $pm}/" | tee -a $D/all.jsonl
    done
  done
done
export MHE_LIB_PATH=$GRAFT_REPO_ROOT/fhe-gpt-2_amd/libmhe.so
for pm in 1 0 1 0; do
  MHE_ROW_PM=$pm step bench_pm$pm 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_pm$pm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pm $pm', d['value'], d['ms_per_step'])" | tee -a $D/bench.txt
done
