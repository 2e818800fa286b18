# r05i: default bench with device memory traced through the ResNet leg; resnet_test 3 x 8 standalone
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05i_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
timeout -k 10 900 python -u bench.py --no-cpu > $D/bench.log 2>&1; echo "bench rc=$?"
grep '^{' $D/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['resnet20']; print(d['value'], r['images_per_s'], r['sec_per_image_1stream'], r['batch_wall_s'], r['scratch_GB'], r['device_mem_used_GB'])"
P=tests/golden/resnet/resnet20_params.bin; C=tests/golden/comp
MHE_RESNET_FIBERS=8 timeout -k 10 300 ./build/resnet_test $P $C 24 20 3 > $D/t3_f8.log 2>&1; echo "t3f8 rc=$? $(grep '^batch:' $D/t3_f8.log)"
