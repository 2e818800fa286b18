# r05zi: the default bench line at the round-5 HEAD (after the encoder FFT tail pass), and rocprofv3 kernel
# bench on one stream (the roofline's per-launch durations)
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r05zi_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > $D/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' $D/bench.log > $D/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$D/hm -o hm --output-format csv -- python3 $R/bench.py --no-cpu --streams 1 --steps 3 --warmup 1 --resnet-images 0 > $D/hm.log 2>&1 || exit $?
find $D/hm -name "*kernel_trace*" -delete
