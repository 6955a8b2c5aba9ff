# Resumed overflow extensions: alignment parity (C3v config included), then C3/C3v A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or simulated_parity or C3_correctness or isoform_rich or C2" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/par.log | head -20; exit $rc; }
bash scripts/gpu_ab_env.sh C3v "RC_RESUME=1" "RC_RESUME=0" || exit 1
bash scripts/gpu_ab_env.sh C3 "RC_RESUME=1"
