# Round 4 (c): tiles (split b chunks reusing their index + DUST masks) and
# shard tests, the C5 rank-2 shard, then the whole C5s job (C5 at the
# mutation rate that keeps ideal 128-cliques) end to end to its matrix.
# Each step under its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r04_c
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "tiles or shards or C4" > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --shard 2/8 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/C5_shard2of8_bench.json 2> $D/C5_shard.err
rc=$?; echo "C5 shard rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/C5_shard.err; exit $rc; }
python3 -c "import json; d=json.load(open('$D/C5_shard2of8_bench.json')); p=d['phases_ms']; print('C5 s2', d['s_per_step'], {k: p[k] for k in ('index_ms','dust_ms','seed_kernel_ms','align_kernel_ms','index_reused','tiles')})"
# slide-read prefetch A/B at C3 (librcgpu_pf.so: -DRC_SLIDE_PREFETCH=1)
for i in 1 2; do
  for v in base pf; do
    L=rna_clique_amd/librcgpu.so; [ $v = pf ] && L=rna_clique_amd/librcgpu_pf.so
    RC_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_$v$i.json 2> $D/C3_$v$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "C3 $v rc=$rc"; tail -5 $D/C3_$v$i.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$D/C3_$v$i.json')); p=d['phases_ms']; print('$v', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'])"
  done
done
timeout -k 10 700 python -u scripts/c5_full.py --config C5s --out $D/c5s_full.json > $D/c5s_full.log 2>&1
rc=$?; echo "C5s full rc=$rc"; tail -4 $D/c5s_full.log
exit $rc
