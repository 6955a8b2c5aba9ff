# C3v kernel stats with and without the 64-lane overflow pass (RC_WIDE=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 0 1; do
  RC_WIDE=$w timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_C3v_w$w -o run -- python3 bench.py --config C3v --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_C3v_w$w.log 2>&1 || exit 1
  echo "== RC_WIDE=$w"; tail -c 1500 gpurun_out/prof_C3v_w$w.log | grep -o '"phases_ms".*' | head -c 900; echo
  f=$(find gpurun_out/prof_C3v_w$w -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e6:9.3f} avg  {r["Name"][:80]}')
PY
done
