# Round 4: windowed row staging -- the -m gpu suite, then the C5 rank-2
# shard (transcripts up to 5 kb: every candidate on the row kernels) and a C3
# bench line. Each step under its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r04_win
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --shard 2/8 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/C5_shard2of8_bench.json 2> $D/C5_shard.err
rc=$?; echo "C5 shard rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/C5_shard.err; exit $rc; }
python3 -c "import json; d=json.load(open('$D/C5_shard2of8_bench.json')); p=d['phases_ms']; print('C5 s2', d['s_per_step'], {k: p[k] for k in ('index_ms','dust_ms','seed_kernel_ms','align_kernel_ms','ext_deferred','ext_wide','defer_length')})"
timeout -k 10 600 python bench.py --config C3 --steps 10 --warmup 2 > $D/C3_bench.json 2> $D/C3_bench.err
rc=$?; echo "C3 bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/C3_bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('$D/C3_bench.json')); print('C3', d['value'], d['ms_per_step'], d['cpu_baseline'])"
