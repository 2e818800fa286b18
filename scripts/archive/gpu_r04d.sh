# r04d: ResNet-20 batch throughput: 4 streams (one image per thread) vs Lockstep threads vs FiberBatch
# (images as fibers on one thread), wall per batch; then rocprofv3 kernel time of 4 batch images
# (8- minus 4-image run) for streams and fibers
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04d
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
run() { # name env... -- args
  local name=$1; shift
  env "$@" MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 300 ./build/resnet_test $P $C $RN_ARGS > gpurun_out/r04d/$name.log 2>&1
}
RN_ARGS="8 20 4" run streams4 MHE_RESNET_FIBERS=1 || exit $?
RN_ARGS="8 20 1" run fibers4 MHE_RESNET_FIBERS=4 || exit $?
RN_ARGS="8 20 1" run fibers8 MHE_RESNET_FIBERS=8 || exit $?
RN_ARGS="8 20 2" run fibers4x2 MHE_RESNET_FIBERS=4 || exit $?
RN_ARGS="8 20 4" run lockstep4 MHE_RESNET_LOCKSTEP=1 || exit $?
for v in "streams 4 1" "fibers 1 4"; do
  set -- $v
  for im in 4 8; do
    d="$R/gpurun_out/r04d/prof_$1_im${im}"
    mkdir -p "$d"
    MHE_RESNET_FIBERS=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o rn --output-format csv -- "$R/build/resnet_test" $P $C $im 20 $2 > "$d/rn.log" 2>&1 || exit $?
    find "$d" -name "*kernel_trace*" -delete
  done
done
