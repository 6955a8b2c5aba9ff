# Round 4 final validation, part 1: smoke + every -m gpu test (one process),
# each under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${R04_TAG:-r04_final}
mkdir -p $D
rocm-smi --showproductname > $D/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; exit $rc
