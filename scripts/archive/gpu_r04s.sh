# r04s: ResNet-20 8-image fiber batches (2 threads x 4 fibers), hoisted rotations on / off alternated:
# an intermittent wrong image was seen once with hoisting on
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04s
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
for v in "h1a 1" "h0a 0" "h1b 1" "h0b 0" "h1c 1" "h0c 0"; do
  set -- $v
  MHE_KS_HOIST=$2 MHE_RESNET_FIBERS=4 timeout -k 10 300 ./build/resnet_test $P $C 8 20 2 > gpurun_out/r04s/$1.log 2>&1
  echo "$1 rc=$?" >> gpurun_out/r04s/rc.txt
done
