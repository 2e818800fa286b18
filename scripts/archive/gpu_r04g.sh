# r04g: kernel time per image in FiberBatch mode (2 threads x 4 fibers): rocprofv3 stats of a 16- minus
# an 8-image batch (both with the same 2-image latency pass)
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for im in 8 16; do
  d="$R/gpurun_out/r04g/prof_f4x2_im${im}"
  mkdir -p "$d"
  MHE_RESNET_FIBERS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o rn --output-format csv -- "$R/build/resnet_test" $P $C $im 20 2 > "$d/rn.log" 2>&1 || exit $?
  find "$d" -name "*kernel_trace*" -delete
done
