# Round 4 (b): parity subset after the slide-loop and seed-order changes, C3
# A/B of the seed kernel's gene order (RC_GENE_ORDER), rocprofv3 kernel stats
# of one C3 step. Each step under its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r04_b
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "simulated_parity or alignment_modes or windowed or C1 or C2 or install" > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for o in 1 0 1 0; do
  RC_GENE_ORDER=$o timeout -k 10 300 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_order$o.json 2> $D/C3_order$o.err || { tail -5 $D/C3_order$o.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/C3_order$o.json')); p=d['phases_ms']; print('order $o', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['index_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_C3 -o run -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $D/prof_C3.log 2>&1
echo "rocprof rc=$?"
