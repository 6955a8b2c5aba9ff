# Index phase changes (fill counts the sort's histograms; DUST after the
# sort's table kernels): sort micro, alignment parity, C3/C3v lines, C3 trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scratch/os_s8 > gpurun_out/os_s8.txt 2>&1; rc=$?; grep -E "n=1600|OK|FAIL" gpurun_out/os_s8.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or simulated_parity or C3_correctness or isoform_rich or C2 or large_index" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/par.log | head -20; exit $rc; }
bash scripts/gpu_ab_env.sh C3 "RC_X=0" || exit 1
bash scripts/gpu_ab_env.sh C3v "RC_X=0" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_C3 -o run -- python3 bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/tr_C3.log 2>&1 && python3 scripts/trace_index.py $(find gpurun_out/tr_C3 -name "*kernel_trace.csv" | head -1) | head -24
