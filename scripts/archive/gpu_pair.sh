# Row-pair 16-bit plane of the packed ModUp intermediate: parity on the new build, then alternating
# HMult bench (ab/libmhe_cur.so = previous build, ab/libmhe_new.so) and one WRITE_SIZE pass each
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pair
cp ab/libmhe_new.so fhe-gpt-2_amd/libmhe.so || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "hmult or switch_key or variants or rotate or prepared" > gpurun_out/pair/pytest.log 2>&1 || exit $?
export TMPDIR=/tmp
for i in 1 2; do
  for v in cur new; do
    cp ab/libmhe_$v.so fhe-gpt-2_amd/libmhe.so || exit 1
    timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 > gpurun_out/pair/b_${v}_$i.json 2>/dev/null || exit $?
    echo "$v $i $(grep -o '"value": [0-9.]*' gpurun_out/pair/b_${v}_$i.json) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/pair/b_${v}_$i.json) $(grep -o '"modup_col_avg_launch_us": [0-9.]*' gpurun_out/pair/b_${v}_$i.json)" >> gpurun_out/pair/summary.txt
  done
done
for v in cur new; do
  cp ab/libmhe_$v.so fhe-gpt-2_amd/libmhe.so || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "^(k_|void k_)" -d "$GRAFT_REPO_ROOT/gpurun_out/pair/pmc_$v" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --resnet-images 0 --streams 1 --steps 1 --warmup 0 --batch 2 > gpurun_out/pair/pmc_$v.log 2>&1 || exit $?
  python3 - $v >> gpurun_out/pair/summary.txt <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
tot = collections.defaultdict(float); ids = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/pair/pmc_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("<")[0].replace("void ", "")
        if k in ("k_modup_col", "k_ks_row_mac"):
            tot[k] += float(r["Counter_Value"]) * 1024; ids[k].add(r.get("Dispatch_Id"))
print(f"{v} WRITE GB per launch: " + ", ".join(f"{k} {tot[k] / max(len(ids[k]), 1) / 1e9:.3f}" for k in sorted(tot)))
PY
  find gpurun_out/pair/pmc_$v -name "*.csv" -delete
done
cp ab/libmhe_new.so fhe-gpt-2_amd/libmhe.so
