# A/B of DUST's whole-wave event threshold (RC_DUST_HEAVY 2 / 4 / 6 / 12 builds; a first run compared 6 / 12 / 24):
# mask parity for each build, then C3v and C3; and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in librcgpu_h2.so librcgpu_h4.so; do
  env RC_LIB=$GRAFT_REPO_ROOT/rna_clique_amd/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dust_mask or degenerate" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/par_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -1 gpurun_out/par_$v.log; [ $rc -eq 0 ] || exit $rc
done


for cfg in C3v C3; do
  for v in librcgpu_h2.so librcgpu_h4.so librcgpu_h6.so librcgpu.so librcgpu_h2.so librcgpu_h4.so librcgpu_h6.so librcgpu.so; do
    env RC_LIB=$GRAFT_REPO_ROOT/rna_clique_amd/$v timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/lab.json 2> gpurun_out/lab.err || { tail -3 gpurun_out/lab.err; exit 1; }
    python scripts/ab_line.py gpurun_out/lab.json "$cfg $v"
  done
done
