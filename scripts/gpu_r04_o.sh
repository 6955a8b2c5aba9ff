# Round 4 (o): seed kernel with the isoform item prefix from the host table
# (no serial prefix loop, one barrier less), no mask load after the last pass,
# candidate ranks counted four samples per dword: parity, A/B against the
# previous commit (librcgpu_prev.so), and the block-cycle split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_o
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C3v; do
  reps=2; [ $cfg = C3v ] && reps=1
  for i in $(seq 1 $reps); do
    for v in prev new; do
      L=rna_clique_amd/librcgpu.so; [ $v != new ] && L=rna_clique_amd/librcgpu_$v.so
      RC_LIB=$L timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D/${cfg}_$v$i.json 2> $D/${cfg}_$v$i.err
      rc=$?; [ $rc -eq 0 ] || { echo "$cfg $v rc=$rc"; tail -5 $D/${cfg}_$v$i.err; exit $rc; }
      python3 -c "import json; d=json.load(open('$D/${cfg}_$v$i.json')); p=d['phases_ms']; print('$cfg $v', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['index_ms'])"
    done
  done
done
RC_LIB=rna_clique_amd/librcgpu_timing.so timeout -k 10 200 python bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_timing.json 2> $D/C3_timing.err
rc=$?; echo "C3 timing rc=$rc"; grep -a "block-cycles" $D/C3_timing.err; exit $rc
