# First sort pass generating its keys from the sequence: micro, parity (large
# index included), then C3/C3v A/B against the written entry array (RC_GEN=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./scratch/os_s8 > gpurun_out/os_s8.txt 2>&1; rc=$?; grep -E "n=1600|OK|FAIL" gpurun_out/os_s8.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or simulated_parity or C3_correctness or isoform_rich or C2 or large_index or dust" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/par.log | head -20; exit $rc; }
bash scripts/gpu_ab_env.sh C3 "RC_GEN=1" "RC_GEN=0" "RC_GEN=1" "RC_GEN=0" || exit 1
bash scripts/gpu_ab_env.sh C3v "RC_GEN=1" "RC_GEN=0"
