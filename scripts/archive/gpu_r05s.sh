# r05s: kernel stats at HEAD -- the HMult bench on one stream and the rescale / key-switch ops at 25 limbs
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05s_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$D/hm -o hm --output-format csv -- python3 $R/bench.py --no-cpu --streams 1 --steps 3 --warmup 1 --resnet-images 0 > $D/hm.log 2>&1 || exit $?
find $D/hm -name "*kernel_trace*" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/ops -o ops --output-format csv -- python3 $R/scripts/ubench_ops.py --limbs 25 --ops rescale8,ks4s --reps 20 > $D/ops.log 2>&1 || exit $?
find $D/ops -name "*kernel_trace*" -delete
