# Kernel trace of one C3 step (rocprofv3 --kernel-trace --stats) and a
# per-launch timeline of the step. Usage: bash scripts/gpu_trace.sh [config] [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-C3}
TAG=${2:-t}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --config "$CFG" --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/trace_timeline.py gpurun_out/prof_$TAG > gpurun_out/timeline_$TAG.txt
tail -60 gpurun_out/timeline_$TAG.txt
