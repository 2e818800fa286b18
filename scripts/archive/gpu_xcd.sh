# XCD-aware ModUp column-pass grid (MHE_MODUP_XCD=1, default) vs the plain mapping: parity, then
# alternating bench runs on one box (both legs), then one FETCH_SIZE pass per mapping
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xcd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "hmult or switch_key or variants or rotate or prepared" > gpurun_out/xcd/pytest.log 2>&1 || exit $?
for i in 1 2; do
  for x in 0 1; do
    MHE_MODUP_XCD=$x timeout -k 10 400 python bench.py --no-cpu --steps 10 --resnet-images 4 > gpurun_out/xcd/b_x${x}_$i.json 2>/dev/null || exit $?
    python3 - $x $i >> gpurun_out/xcd/summary.txt <<'PY'
import json, sys
x, i = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f"gpurun_out/xcd/b_x{x}_{i}.json") if l.startswith("{")][-1])
r = d["resnet20"]
print(f"xcd={x} run={i} HMult/s={d['value']} row_mac_us={d['roofline']['avg_launch_us']} modup_col_us={d['roofline']['modup_col_avg_launch_us']} resnet_s={r['sec_per_image_1stream']} images_per_s={r['images_per_s']}")
PY
  done
done
export TMPDIR=/tmp
for x in 0 1; do
  MHE_MODUP_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "^(k_|void k_)" -d "$GRAFT_REPO_ROOT/gpurun_out/xcd/pmc$x" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --resnet-images 0 --streams 1 --steps 1 --warmup 0 --batch 2 > gpurun_out/xcd/pmc$x.log 2>&1 || exit $?
  python3 - $x >> gpurun_out/xcd/summary.txt <<'PY'
import csv, glob, sys, collections
x = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob(f"gpurun_out/xcd/pmc{x}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("<")[0].replace("void ", "")
        if k in ("k_modup_col", "k_ks_row_mac"):
            tot[k] += float(r["Counter_Value"]) * 2048; n[k] += 1
print(f"xcd={x} FETCH x2 GB per launch: " + ", ".join(f"{k} {tot[k] / max(n[k], 1) / 1e9:.3f}" for k in sorted(tot)))
PY
  find gpurun_out/xcd/pmc$x -name "*.csv" -delete
done
