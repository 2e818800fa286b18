# r06m: kernel trace of 8 batched rescales at 25 limbs (scripts/ubench_ops.py rescale8): per-kernel
# durations and the gaps between them
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
D=gpurun_out/r06m_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/rs -o rs --output-format csv -- python3 $R/scripts/ubench_ops.py --limbs 25 --ops rescale8,rescale --reps 30 > $D/rs.log 2>&1 || exit $?
grep '^{' $D/rs.log
