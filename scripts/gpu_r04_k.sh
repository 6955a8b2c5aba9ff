# Round 4 (k): row kernel with a wave-uniform slide loop (one ballot per
# round, no exec-mask bookkeeping) and the row-step count taken from the
# extensions' step counters instead of every step, the step's room from a
# per-extension constant, the gap state's E bits set after the slide: parity, A/B against the
# previous commit (librcgpu_prev.so) and the same sources without the uniform
# loop (librcgpu_su0.so), and the row kernel's instruction mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_k
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C3v; do
  reps=2; [ $cfg = C3v ] && reps=1
  for i in $(seq 1 $reps); do
    for v in prev new su0; do
      L=rna_clique_amd/librcgpu.so; [ $v != new ] && L=rna_clique_amd/librcgpu_$v.so
      RC_LIB=$L timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D/${cfg}_$v$i.json 2> $D/${cfg}_$v$i.err
      rc=$?; [ $rc -eq 0 ] || { echo "$cfg $v rc=$rc"; tail -5 $D/${cfg}_$v$i.err; exit $rc; }
      python3 -c "import json; d=json.load(open('$D/${cfg}_$v$i.json')); p=d['phases_ms']; print('$cfg $v', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['ext_steps'])"
    done
  done
done
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "extend_rows" --output-format csv -d $D/pmc/p1 -o run -- python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/pmc_p1.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_scale.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/gpu_tests2.log 2>&1
rc=$?; echo "pytest2 rc=$rc"; tail -3 $D/gpu_tests2.log; exit $rc
