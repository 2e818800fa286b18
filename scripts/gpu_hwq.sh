# HIP hardware-queue count vs stream count: ResNet-20 batch and HMult bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 ./build/resnet_test $P $C 8 20 8 > gpurun_out/hwq8_s8.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 ./build/resnet_test $P $C 8 20 6 > gpurun_out/hwq8_s6.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --streams 8 > gpurun_out/hwq8_b8.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --streams 4 > gpurun_out/hwq8_b4.log 2>&1 || exit $?
