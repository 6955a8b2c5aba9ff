# Quick iteration: GPU parity tests, then the bench without the CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config "${1:-C3}" --steps "${2:-3}" --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc=$rc"
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'],d['ms_per_step']);print(d['phases_ms'])"
exit $rc
