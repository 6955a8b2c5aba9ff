# 16-lane sliding rows (RC_ROW_WIDTH=16) in the shared-search path: parity, then C3/C3v A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RC_ROW_WIDTH=16 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or simulated_parity or C3_correctness or isoform_rich or C2" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par16.log 2>&1
rc=$?; echo "parity16 rc=$rc"; tail -2 gpurun_out/par16.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/par16.log | head -10; }
bash scripts/gpu_ab_env.sh C3 "RC_ROW_WIDTH=32" "RC_ROW_WIDTH=16" || exit 1
for cfg in C3 C3v; do RC_ROW_WIDTH=16 timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab16_$cfg.json 2>/dev/null && python -c "import json; p=json.load(open('gpurun_out/ab16_$cfg.json'))['phases_ms']; print('$cfg', {k: p.get(k) for k in ('total_ms','align_kernel_ms','ext_fullband','ext_slides','ext_wide','ext_deferred','ext_steps')})"; done
bash scripts/gpu_ab_env.sh C3v "RC_ROW_WIDTH=16"
