# Same-box A/B of libmhe builds (ab/libmhe_<v>.so) on both bench legs: each variant is copied over
# the snapshot's libmhe.so (libmhe_seal.so links it by path), C2 parity first, then bench.py
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sw
for v in ${VARIANTS:-cur occ3 dpf0 cur}; do
  cp "ab/libmhe_$v.so" fhe-gpt-2_amd/libmhe.so || exit 1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "hmult_c2 or n16_variants or switch_key_inplace" > gpurun_out/sw/pytest_$v.log 2>&1 || exit $?
  timeout -k 10 400 python bench.py --no-cpu --steps 10 --resnet-images 4 > gpurun_out/sw/bench_$v.json 2>/dev/null || exit $?
  python3 - "$v" >> gpurun_out/sw/summary.txt <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/sw/bench_{v}.json") if l.startswith("{")][-1])
r = d["resnet20"]
print(v, d["value"], d["roofline"]["avg_launch_us"], d["roofline"].get("modup_col_avg_launch_us"),
      r["sec_per_image_1stream"], r["bootstrap_s_per_image"], r["images_per_s"])
PY
done
cp ab/libmhe_cur.so fhe-gpt-2_amd/libmhe.so
