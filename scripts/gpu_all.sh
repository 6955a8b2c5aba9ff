# GPU tests, smoke, then bench + rocprof. Stops at the first GPU fault/abort/timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_check.sh
rc=$?
echo "check rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench.sh "${1:-C3}" "${2:-3}"
