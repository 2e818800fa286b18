# r04s: ResNet-20 8-image batch modes with hoisted rotations: threads x fibers 2x4, 1x8, 4x2, 2x4
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04s
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "f4x2a 2 4" "f8x1 1 8" "f2x4 4 2" "f4x2b 2 4"; do
  set -- $v
  MHE_RESNET_FIBERS=$3 timeout -k 10 300 ./build/resnet_test $P $C 8 20 $2 > gpurun_out/r04s/$1.log 2>&1 || exit $?
done
