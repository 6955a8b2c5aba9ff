# Cooperative-DUST check: micro variants (random / poly-A), then the DUST mask
# parity test and the alignment parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_dust.sh "$@" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dust or alignment_modes or isoform_rich" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par_dust.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/par_dust.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/par_dust.log | head -20; exit $rc; }
