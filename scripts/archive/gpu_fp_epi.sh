# FP64 ModDown / rescale epilogues: the full parity file and the SEAL-surface tests on the new build,
# then alternating bench runs (both legs) of ab/libmhe_cur.so and ab/libmhe_new.so
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/epi
cp ab/libmhe_new.so fhe-gpt-2_amd/libmhe.so || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -x -q --timeout 300 --timeout-method thread > gpurun_out/epi/pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_seal_api.py -m gpu -x -q --timeout 400 --timeout-method thread -k "seal_api_end_to_end or resnet20 or bootstrapping" > gpurun_out/epi/pytest_seal.log 2>&1 || exit $?
for i in 1 2; do
  for v in cur new; do
    cp ab/libmhe_$v.so fhe-gpt-2_amd/libmhe.so || exit 1
    timeout -k 10 400 python bench.py --no-cpu --steps 10 --resnet-images 4 > gpurun_out/epi/b_${v}_$i.json 2>/dev/null || exit $?
    python3 - $v $i >> gpurun_out/epi/summary.txt <<'PY'
import json, sys
v, i = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f"gpurun_out/epi/b_{v}_{i}.json") if l.startswith("{")][-1])
r = d["resnet20"]
print(f"{v} run={i} HMult/s={d['value']} row_mac_us={d['roofline']['avg_launch_us']} resnet_s={r['sec_per_image_1stream']} boot_s={r['bootstrap_s_per_image']} images_per_s={r['images_per_s']}")
PY
  done
done
cp ab/libmhe_new.so fhe-gpt-2_amd/libmhe.so
