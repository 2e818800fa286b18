# ResNet-20 leg: images in flight (host threads / HIP streams) x images per batch, same box
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rs
for cfg in "4 4" "8 4" "8 8" "6 6" "4 4"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --no-cpu --steps 2 --warmup 1 --resnet-images $1 --resnet-streams $2 > gpurun_out/rs/i$1_s$2.json 2>/dev/null || exit $?
  python3 - $1 $2 >> gpurun_out/rs/summary.txt <<'PY'
import json, sys
i, s = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f"gpurun_out/rs/i{i}_s{s}.json") if l.startswith("{")][-1])
r = d["resnet20"]
print(f"images={i} streams={s} images_per_s={r['images_per_s']} batch_wall_s={r['batch_wall_s']} s_per_image_1stream={r['sec_per_image_1stream']}")
PY
done
