# r03t: round evidence at HEAD -- the whole GPU suite, smoke, the default bench line, rocprofv3
# kernel-trace stats of the HMult leg and its PMC traffic (scripts/gpu_round.sh), then the GPT-2
# block at GPT-2 width (scripts/gpu_gpt2_full.sh).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r03t bash scripts/gpu_round.sh || exit $?
FULL_LIMIT=700 bash scripts/gpu_gpt2_full.sh || exit $?
