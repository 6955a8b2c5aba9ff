# Quick iteration: GPU parity tests, then the bench without the CPU baseline.
# Usage: bash scripts/gpu_quick.sh [config] [steps] [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
K=${3:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config "${1:-C3}" --steps "${2:-3}" --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc=$rc"
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'],d['ms_per_step']);print(d['phases_ms']);print(d['graph'])"
exit $rc
