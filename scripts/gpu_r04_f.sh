# Round 4 (f): DUST masks made once per sample across ranks (tests; the
# 8-rank C3 shard times with --share-dust), and a seed-kernel occupancy A/B
# (librcgpu_s5.so: 512-seed LDS passes at 5 waves/SIMD; librcgpu_c512.so:
# 512-seed passes alone).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_f
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "dust or sharded or tiles" > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/shard_time.py --config C3 --shards 8 --reps 2 --share-dust > $D/C3_shards8_sharedust.txt 2>&1
rc=$?; echo "shards rc=$rc"; grep shard $D/C3_shards8_sharedust.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base s5 c512; do
    L=rna_clique_amd/librcgpu.so; [ $v != base ] && L=rna_clique_amd/librcgpu_$v.so
    RC_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_$v$i.json 2> $D/C3_$v$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "C3 $v rc=$rc"; tail -5 $D/C3_$v$i.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$D/C3_$v$i.json')); p=d['phases_ms']; print('$v', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['index_ms'])"
  done
done
exit 0
