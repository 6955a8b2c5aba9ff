# Run the onesweep micro variants (built on the CPU side into scratch/), then
# a rocprofv3 kernel-stats pass over the first one. Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in "$@"; do
  echo "== $b"
  timeout -k 10 120 ./scratch/$b > gpurun_out/$b.txt 2>&1 || { cat gpurun_out/$b.txt; exit 1; }
  cat gpurun_out/$b.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_os -o run -- ./scratch/$1 > gpurun_out/prof_os.log 2>&1 || exit 1
f=$(find gpurun_out/prof_os -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e6:9.3f} avg  {r["Name"][:100]}')
PY
