# r04q: fused key MAC digit loop with fixed load shapes (counted waits): key-switch parity, the bench's
# timed path, then HMult/s A/B against the previous library on the same box (old, new, old, new)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04q
rm -f gpurun_out/r04q/ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_bench_path.py -m gpu -x -q --timeout 580 --timeout-method thread > gpurun_out/r04q/tests.log 2>&1 || exit $?
for v in old new old new; do
  if [ $v = old ]; then export MHE_LIB_PATH=build/var/old/libmhe.so; else unset MHE_LIB_PATH; fi
  timeout -k 10 200 python bench.py --no-cpu --resnet-images 0 --steps 20 --warmup 5 > gpurun_out/r04q/b_$v.log 2>&1 || exit $?
  echo "{\"lib\": \"$v\", \"line\": $(tail -n 1 gpurun_out/r04q/b_$v.log)}" >> gpurun_out/r04q/ab.jsonl
done
