# Round-3 re-measurement after the DUST threshold change (RC_DUST_HEAVY 6):
# smoke + the whole GPU suite, the bench line at the driver's settings,
# rocprofv3 kernel stats of one C3 step, the PMC passes, C3v and C4 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit 1
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/C3_bench.json 2> gpurun_out/final/C3_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/final/C3_bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/final/C3_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'), d['wall_clock_to_matrix']['wall_clock_s'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_C3 -o run -- python3 bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/final/prof_C3.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh C3 || exit 1
for cfg in C3v C4; do
  timeout -k 10 600 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/final/${cfg}_bench.json 2> gpurun_out/final/${cfg}_bench.err || { echo "bench $cfg failed"; tail -3 gpurun_out/final/${cfg}_bench.err; exit 1; }
  python scripts/ab_line.py gpurun_out/final/${cfg}_bench.json "$cfg"
done
exit 0
