# r06y: the default bench line at HEAD with the ResNet batch at 4 x 8
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06y_$(date +%H%M%S)
mkdir -p $D
echo "logs in $D"
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > $D/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' $D/bench.log > $D/bench.json; exit $rc
