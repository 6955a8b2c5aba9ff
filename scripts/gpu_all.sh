# Every GPU test in one call: smoke, the -m gpu suite without the scale tests,
# then the scale tests (C4 8-shard emulation, C5 rank shard). Each step under
# its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_scale.py > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 650 --timeout-method thread -p no:cacheprovider > gpurun_out/scale_tests.log 2>&1
rc=$?; echo "scale tests rc=$rc"; tail -15 gpurun_out/scale_tests.log
exit $rc
