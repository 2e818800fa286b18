# r06l: hardware queues per process (GPU_MAX_HW_QUEUES, the box's default 4) against HIP streams:
# HMult bench at 4 / 6 / 8 streams, ResNet-20 batch at 3 x 8 and 4 x 8.
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06l_$(date +%H%M%S)
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
hm() { grep '^{' $D/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['modup_col_avg_launch_us'])" | tee -a $D/bench.txt; }
step hm_q4_s4 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3 --streams 4; hm hm_q4_s4
GPU_MAX_HW_QUEUES=8 step hm_q8_s4 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3 --streams 4; hm hm_q8_s4
GPU_MAX_HW_QUEUES=8 step hm_q8_s6 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3 --streams 6; hm hm_q8_s6
GPU_MAX_HW_QUEUES=8 step hm_q8_s8 300 python -u bench.py --resnet-images 0 --no-cpu --steps 20 --warmup 3 --streams 8; hm hm_q8_s8
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
LD_LIBRARY_PATH=fhe-gpt-2_amd MHE_RESNET_FIBERS=8 step rn_q4_3x8 400 ./build/resnet_test $P $C 24 20 3
echo "rn_q4_3x8 $(grep '^batch:' $D/rn_q4_3x8.log)" | tee -a $D/resnet.txt
GPU_MAX_HW_QUEUES=8 LD_LIBRARY_PATH=fhe-gpt-2_amd MHE_RESNET_FIBERS=8 step rn_q8_3x8 400 ./build/resnet_test $P $C 24 20 3
echo "rn_q8_3x8 $(grep '^batch:' $D/rn_q8_3x8.log)" | tee -a $D/resnet.txt
GPU_MAX_HW_QUEUES=8 LD_LIBRARY_PATH=fhe-gpt-2_amd MHE_RESNET_FIBERS=8 step rn_q8_4x8 500 ./build/resnet_test $P $C 32 20 4
echo "rn_q8_4x8 $(grep '^batch:' $D/rn_q8_4x8.log)" | tee -a $D/resnet.txt
