# r06g: wave-local ModUp column transposes with plain (not non-temporal) intermediate stores
# (build/vx/wavent: MHE_MODUP_WAVE=1 MHE_NT=4) against main and build/vx/nt4 (MHE_NT=4 alone).
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06g_$(date +%H%M%S)
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
MHE_LIB_PATH=$R/build/vx/wavent/libmhe.so step parity_wavent 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_bench_path.py
tail -1 $D/parity_wavent.log
for rep in 1 2; do
for lib in main wavent nt4; do
  if [ $lib = main ]; then L=$R/fhe-gpt-2_amd/libmhe.so; else L=$R/build/vx/$lib/libmhe.so; fi
  MHE_LIB_PATH=$L step bench_${lib}_$rep 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3
  grep '^{' $D/bench_${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['modup_col_avg_launch_us'], d.get('valu_roofline',{}).get('frac'))" | tee -a $D/bench.txt
done
done
