# A/B of the current libmhe.so against build/ab/base/libmhe.so on one box: HMult bench line
# (bench.py, no CPU / ResNet legs) and the logn-14 bootstrap (boot_test), alternating, after a
# quick parity pass of the current library.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q -k "${PYK:-extreme or switch_key or hmult or rotate or rescale or batch}" --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export MHE_LIB_PATH="$PWD/build/ab/base/libmhe.so"; export LD_LIBRARY_PATH="$PWD/build/ab/base"; else unset MHE_LIB_PATH; unset LD_LIBRARY_PATH; fi
    timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps ${STEPS:-20} --warmup 3 > gpurun_out/ab/hm_${v}_$rep.json 2>gpurun_out/ab/hm_${v}_$rep.err || exit $?
    timeout -k 10 300 ./build/boot_test 14 3 > gpurun_out/ab/boot_${v}_$rep.log 2>&1 || exit $?
  done
done
unset MHE_LIB_PATH LD_LIBRARY_PATH
python3 - <<'PY'
import json, glob, re
for f in sorted(glob.glob("gpurun_out/ab/hm_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["roofline"]["avg_launch_us"], d["roofline"]["modup_col_avg_launch_us"])
for f in sorted(glob.glob("gpurun_out/ab/boot_*.log")):
    t = re.findall(r"bootstrap \d: ([0-9.]+) s", open(f).read())
    print(f, t)
PY
