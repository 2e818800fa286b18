# r04d: kernel time of 4 batch images, 4 streams vs Lockstep (rocprofv3 stats of an 8- minus a 4-image
# batch run; both also run the same 2-image latency pass)
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for ls in 0 1; do
  for im in 4 8; do
    d="$R/gpurun_out/r04d_ls${ls}_im${im}"
    mkdir -p "$d"
    MHE_RESNET_LOCKSTEP=$ls MHE_RESNET_LOCKSTEP_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o rn --output-format csv -- "$R/build/resnet_test" $P $C $im 20 4 > "$d/rn.log" 2>&1 || exit $?
    find "$d" -name "*kernel_trace*" -delete
  done
done
