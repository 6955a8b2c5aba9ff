# Bench + rocprof on one GPU. Usage: bash scripts/gpu_bench.sh [config] [steps]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=${1:-C3}
STEPS=${2:-3}
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1 || true
timeout -k 10 900 python bench.py --config "$CFG" --steps "$STEPS" --warmup 1 > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$CFG.json
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o run -- python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/prof_$CFG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
