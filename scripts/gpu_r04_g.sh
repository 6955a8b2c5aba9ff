# Round 4 (g): seed kernel with fewer dependent round trips per gene (one-load
# position -> transcript records, contiguous isoform records, k-mer / window /
# bucket loads beside the DUST test, slot claims under the sort) -- parity
# suite, then A/B against the previous commit's library (librcgpu_prev.so)
# and the same sources at 5 waves/SIMD with 512-seed passes (librcgpu_s5.so);
# the 8-rank C3 shard times with DUST masks shared (the mask pass now reuses
# the shard's own tile).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_g
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in prev new s5; do
    L=rna_clique_amd/librcgpu.so; [ $v = prev ] && L=rna_clique_amd/librcgpu_prev.so; [ $v = s5 ] && L=rna_clique_amd/librcgpu_s5.so
    RC_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_$v$i.json 2> $D/C3_$v$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "C3 $v rc=$rc"; tail -5 $D/C3_$v$i.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$D/C3_$v$i.json')); p=d['phases_ms']; print('$v', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['index_ms'])"
  done
done
timeout -k 10 400 python -u scripts/shard_time.py --config C3 --shards 8 --reps 2 --share-dust > $D/C3_shards8_sharedust.txt 2>&1
rc=$?; echo "shards rc=$rc"; grep shard $D/C3_shards8_sharedust.txt; exit $rc
