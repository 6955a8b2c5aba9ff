# Round 4 (q): the DUST-mask exchange with real engines -- the RCCL device
# path (world 1, forced) in the test suite, and two ranks sharing the GPU over
# gloo through bench.py (the sharded step: masks, alignment, edges, graph);
# then the 8-rank C3 shard times under the refitted planner.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_q
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "rccl or dust or sharded or C4" > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --config C2 --steps 2 --warmup 1 --no-cpu-baseline > $D/C2_gpus2_gloo.json 2> $D/C2_gpus2_gloo.err
rc=$?; echo "bench gpus2 rc=$rc"; tail -c 600 $D/C2_gpus2_gloo.json; [ $rc -eq 0 ] || { tail -20 $D/C2_gpus2_gloo.err; exit $rc; }
timeout -k 10 400 python -u scripts/shard_time.py --config C3 --shards 8 --reps 2 --share-dust > $D/C3_shards8_sharedust.txt 2>&1
rc=$?; echo "shards rc=$rc"; grep shard $D/C3_shards8_sharedust.txt; exit $rc
