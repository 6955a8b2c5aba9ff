# extend_kernel starting searches from the row kernel's first-seed HSP:
# alignment parity (incl. the C3v correctness config), then C3v A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in 0 1; do
RC_WIDE=$w timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or simulated_parity or C3_correctness or isoform_rich or C2" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par_w$w.log 2>&1
rc=$?; echo "parity RC_WIDE=$w rc=$rc"; tail -2 gpurun_out/par_w$w.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/par_w$w.log | head -20; exit $rc; }
done
bash scripts/gpu_ab_env.sh C3v "RC_REUSE=0" "RC_REUSE=1" "RC_WIDE=1" || exit 1
bash scripts/gpu_ab_env.sh C3 "RC_REUSE=1" "RC_WIDE=1"
