set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"
case $rc in 0|1) ;; *) echo "stopping after smoke rc=$rc"; exit $rc;; esac
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
exit $rc
