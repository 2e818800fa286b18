# r05h: C5 at GPT-2 width with the reference's GELU (per-stage errors, s/block, error vs poly.py as
# written), then the default bench line (ResNet batch 3 x 8)
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05h_$(date +%H%M%S)
mkdir -p $D/fx
echo "logs in $D"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py > $D/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $D/parity.log; [ $rc -eq 0 ] || exit $rc
python3 tests/golden/gpt2_block/make_fixture.py --full $D/fx --gelu-ref > /dev/null
timeout -k 10 900 ./build/gpt2_block_test $D/fx block > $D/gpt2_ref.log 2>&1; echo "gpt2_ref rc=$?"
grep -E "stages|GELU x piece|block_seconds|PASS|FAIL" $D/gpt2_ref.log
rm -rf $D/fx
timeout -k 10 900 python -u bench.py > $D/bench.log 2>&1; echo "bench rc=$?"
grep '^{' $D/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['resnet20']; print(d['value'], d['ms_per_step'], r['images_per_s'], r['sec_per_image_1stream'], r['batch_wall_s'], r['scratch_GB'], r['device_mem_used_GB_after_batch'])"
