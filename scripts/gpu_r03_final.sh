# Round-3 measurements on the final sources: the bench line at the driver's
# settings (CPU baseline and wall-clock leg included), rocprofv3 kernel stats
# of one C3 step, the PMC passes, bench lines of the other configs and the C5
# rank-2 shard. Each step under its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
nproc > gpurun_out/final/nproc.txt; lscpu > gpurun_out/final/lscpu.txt 2>&1 || true
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/C3_bench.json 2> gpurun_out/final/C3_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/final/C3_bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/final/C3_bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d.get('cpu_baseline',{}).get('value'), d['wall_clock_to_matrix']['wall_clock_s'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_C3 -o run -- python3 bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/final/prof_C3.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh C3 || exit 1
for cfg in C1 C2 C4 C3v; do
  timeout -k 10 600 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/final/${cfg}_bench.json 2> gpurun_out/final/${cfg}_bench.err || { echo "bench $cfg failed"; tail -3 gpurun_out/final/${cfg}_bench.err; exit 1; }
  python scripts/ab_line.py gpurun_out/final/${cfg}_bench.json "$cfg"
done
timeout -k 10 600 python bench.py --config C5 --shard 2/8 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/final/C5_shard2of8_bench.json 2> gpurun_out/final/C5_shard.err
rc=$?; echo "C5 shard rc=$rc"; tail -c 600 gpurun_out/final/C5_shard2of8_bench.json
exit 0
