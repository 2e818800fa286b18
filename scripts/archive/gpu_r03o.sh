# r03o: ModUp column-pass occupancy (MHE_MODUP_OCC 2: 178 VGPRs no spills / 3: 168 + 12 spills
# (default) / 4: 128 + 58 spills) at ResNet levels and on the C2 HMult leg
# (build/var/{twz,mocc2,mocc4}: bash scripts/build_var.sh mocc2 -DMHE_MODUP_OCC=2, ...).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03o
mkdir -p $O
for lib in twz mocc2 mocc4 twz mocc2 mocc4; do
  export MHE_LIB_PATH="$PWD/build/var/$lib/libmhe.so"
  timeout -k 10 200 python scripts/ubench_ops.py --ops ks,ks4s,rot4,hmult >> $O/ops_$lib.jsonl 2>> $O/ops.err || exit $?
  timeout -k 10 300 python bench.py --no-cpu --resnet-images 0 --steps 10 --warmup 2 > $O/hm_${lib}_$(date +%s).json 2>> $O/ops.err || exit $?
done
