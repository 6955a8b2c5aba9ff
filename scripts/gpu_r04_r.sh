# Round 4 (r): row kernel at 8 waves per SIMD (64 VGPRs, spills only in the
# fetch transition) A/B against the default 7 (librcgpu_w8.so), and the C3 /
# C3v config tests with 20 oracle pairs covering every sample (durations).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${R04_TAG:-r04_r}
mkdir -p $D
for cfg in C3 C3v; do
  reps=2; [ $cfg = C3v ] && reps=1
  for i in $(seq 1 $reps); do
    for v in main w8; do
      L=rna_clique_amd/librcgpu.so; [ $v != main ] && L=rna_clique_amd/librcgpu_$v.so
      RC_LIB=$L timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D/${cfg}_$v$i.json 2> $D/${cfg}_$v$i.err
      rc=$?; [ $rc -eq 0 ] || { echo "$cfg $v rc=$rc"; tail -5 $D/${cfg}_$v$i.err; exit $rc; }
      python3 -c "import json; d=json.load(open('$D/${cfg}_$v$i.json')); p=d['phases_ms']; print('$cfg $v', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['index_ms'])"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "C3" -x -v --durations=0 --timeout 400 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|s call" $D/gpu_tests.log | tail -6; exit $rc
