# Round 4 (j): the full GPU suite with the seed kernel at 5 waves (512-seed
# passes) and the refitted shard planner; C3 bench; the 8-rank C3 shard
# times with shared DUST masks under the new plan.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_j
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C3 --steps 5 --warmup 1 --no-e2e > $D/C3_bench.json 2> $D/C3_bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json; d=json.load(open('$D/C3_bench.json')); p=d['phases_ms']; print(d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['index_ms'], d['roofline'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/shard_time.py --config C3 --shards 8 --reps 2 --share-dust > $D/C3_shards8_sharedust.txt 2>&1
rc=$?; echo "shards rc=$rc"; grep shard $D/C3_shards8_sharedust.txt; exit $rc
