# A/B of two library builds (RC_LIB) and the resume modes on C3 and C3v.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "alignment_modes or C3_correctness or isoform_rich" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C3v; do
  for v in "librcgpu_head.so X=0" "librcgpu.so RC_RESUME=0" "librcgpu.so RC_RESUME=1" "librcgpu.so X=0" "librcgpu_head.so X=0"; do
    set -- $v
    env RC_LIB=$GRAFT_REPO_ROOT/rna_clique_amd/$1 $2 timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/lab.json 2> gpurun_out/lab.err || { tail -3 gpurun_out/lab.err; exit 1; }
    python scripts/ab_line.py gpurun_out/lab.json "$cfg $1 $2"
  done
done
