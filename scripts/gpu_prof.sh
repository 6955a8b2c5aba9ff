# Kernel trace + stats of one bench step (rocprofv3), summary to gpurun_out/prof_<tag>/
# Usage: bash scripts/gpu_prof.sh [config] [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-C3}
TAG=${2:-p}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --config "$CFG" --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e6:9.3f} avg  {r["Name"][:110]}')
PY
exit $rc
