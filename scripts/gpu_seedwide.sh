# A/B of the seed kernel's small-bucket wide load (RC_SEED_WIDE 0 / 8 / 16 builds) on C3 and C3v.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or C3_correctness or isoform_rich or large_index or ambiguous or degenerate or 201" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C3v; do
  for v in librcgpu_w0.so librcgpu.so librcgpu_w16.so librcgpu_w0.so librcgpu.so librcgpu_w16.so; do
    env RC_LIB=$GRAFT_REPO_ROOT/rna_clique_amd/$v timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/lab.json 2> gpurun_out/lab.err || { tail -3 gpurun_out/lab.err; exit 1; }
    python scripts/ab_line.py gpurun_out/lab.json "$cfg $v"
  done
done
