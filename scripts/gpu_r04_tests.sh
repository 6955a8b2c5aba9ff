# Round 4: smoke + the whole -m gpu suite (new: 300 samples, a 4200-isoform
# gene, the graph phase at C5 size), each under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04_tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_tests/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04_tests/smoke.log; exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tests/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r04_tests/gpu_tests.log
exit $rc
