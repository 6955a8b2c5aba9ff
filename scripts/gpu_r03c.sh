# Round-3 checkpoint: alignment parity tests (the index sort is new), a C3
# bench line with every output (no CPU baseline), a C3v kernel-stats profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in os_s8 os_s1 os_s4 os_s16; do echo "== $b"; timeout -k 10 120 ./scratch/$b > gpurun_out/$b.txt 2>&1; rc=$?; grep -E "n=1600|n=2000|OK|FAIL" gpurun_out/$b.txt; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or simulated_parity or C3_correctness or 201 or isoform_rich or C2" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/par.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/par.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_C3.json 2> gpurun_out/bench_C3.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_C3.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_C3.json')); print(d['value'], d['ms_per_step'], d['wall_clock_to_matrix'], d['phases_ms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_C3v -o run -- python3 bench.py --config C3v --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/prof_C3v.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_C3v -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:18]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e6:9.3f} avg  {r["Name"][:90]}')
PY
exit 0
