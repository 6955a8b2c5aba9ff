# Round-end validation on one GPU: smoke + every -m gpu test, the default
# bench line, a rocprofv3 kernel-stats pass and the PMC passes, each step
# under its own time limit; stops at the first failure.
# Usage: bash scripts/gpu_round_end.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_bench.sh C3 10 || exit $?
bash scripts/gpu_pmc.sh C3 || exit $?
