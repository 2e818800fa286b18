# k_icol_lift group size sweep on the ResNet leg (MHE_ICOL_GROUP), against the unfused path.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > gpurun_out/icol2_parity.log 2>&1 || exit $?
: > gpurun_out/icol2_summary.txt
for v in ${ICOL2_VARIANTS:-g1 off g2 g1 off}; do
  if [ "$v" = off ]; then export MHE_ICOL_FUSED=0; unset MHE_ICOL_GROUP; else export MHE_ICOL_FUSED=1 MHE_ICOL_GROUP=${v#g}; fi
  timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/icol2_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"sec_per_image_1stream": [0-9.]*\|"images_per_s": [0-9.]*' gpurun_out/icol2_$v.log | tr '\n' ' ')" >> gpurun_out/icol2_summary.txt
done
