# r06k: why the ping-pong ModUp image is slower: ping (main), noping, ping with the end barrier kept
# (pingbar), noping with the ping image's LDS size (nopingpad).  HMult bench only, 2 rounds.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06k_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $D/rc.txt
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }
}
for rep in 1 2; do
for lib in main noping pingbar nopingpad; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  MHE_LIB_PATH=$L step bench_${lib}_$rep 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['modup_col_avg_launch_us'], d.get('valu_roofline',{}).get('frac'))" | tee -a $D/bench.txt
done
done
