# r03v: output primes per workgroup of the ModDown / rescale lift column pass (MHE_ICOL_GROUP 1
# default / 2 / 3 / 4): each workgroup redoes the special (or last) limb's inverse column stages for
# its group, so larger groups trade redundant work for a narrower grid.  L = 31 and L = 20.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03v
mkdir -p $O
for g in 1 2 3 4 1 2 3 4; do
  for L in 31 20; do
    MHE_ICOL_GROUP=$g timeout -k 10 200 python scripts/ubench_ops.py --limbs $L --ops rescale,rescale4,ks,ks4 --reps 40 | sed "s/}/, \"group\": $g}/" >> $O/sweep.jsonl 2>> $O/err.log || exit $?
  done
done
