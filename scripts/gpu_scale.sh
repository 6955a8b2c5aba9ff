# Scale checks on one GPU: the C4 8-shard emulation and the C5 rank shard
# tests, the C5 rank-2 shard bench, and bench.py --gpus 2 (ranks launched by
# bench.py itself, gloo on one GPU). Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -n "$SKIP_SCALE_TESTS" ] || timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 650 --timeout-method thread -p no:cacheprovider > gpurun_out/scale_tests.log 2>&1
rc=$?; echo "scale tests rc=$rc"; tail -15 gpurun_out/scale_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config C5 --shard 2/8 --steps 1 --warmup 0 > gpurun_out/c5_shard.json 2> gpurun_out/c5_shard.err
rc=$?; echo "c5 shard rc=$rc"; tail -c 2500 gpurun_out/c5_shard.json; tail -5 gpurun_out/c5_shard.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --gpus 2 --steps 2 --warmup 1 --config C2 --backend gloo --no-cpu-baseline > gpurun_out/bench_gpus2.json 2> gpurun_out/bench_gpus2.err
rc=$?; echo "gpus2 rc=$rc"; tail -c 2500 gpurun_out/bench_gpus2.json; tail -5 gpurun_out/bench_gpus2.err
exit $rc
