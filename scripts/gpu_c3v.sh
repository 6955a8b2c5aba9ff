# Row-kernel change check: C3 and C3v quick benches, then the alignment parity
# tests (indels, minus strand, poly-A) and the C3v config test.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in C3 C3v; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab_$cfg.json 2> gpurun_out/ab_$cfg.err || { echo "bench $cfg failed"; tail -5 gpurun_out/ab_$cfg.err; exit 1; }
  python scripts/ab_line.py gpurun_out/ab_$cfg.json "$cfg"
  python -c "import json; p=json.load(open('gpurun_out/ab_$cfg.json'))['phases_ms']; print({k: p[k] for k in ('ext_fullband','ext_slides','ext_wide','ext_deferred','ext_calls','align_ms','band_bound')})"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or simulated_parity or C3_correctness or 201 or isoform_rich or C2" -p no:cacheprovider > gpurun_out/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/par.log
exit $rc
