# Round 4 (w): the whole -m gpu suite as the driver runs it (one process,
# -q), with per-test durations: its wall time after the config tests'
# oracle sample went to 12 pairs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${R04_TAG:-r04_w}
mkdir -p $D
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --durations=15 -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -22 $D/gpu_tests.log; exit $rc
