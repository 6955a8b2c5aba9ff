# Multi-process rehearsal on one GPU: GPU tests (incl. the 2-process shard
# test), then bench.py under torch.distributed.run with 2 ranks sharing the
# GPU over gloo (RCCL needs one GPU per rank; the driver's N-GPU runs use it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --config "${1:-C2}" --backend gloo > gpurun_out/bench_dist.json 2> gpurun_out/bench_dist.err
rc=$?; echo "dist bench rc=$rc"; tail -c 1500 gpurun_out/bench_dist.json; tail -5 gpurun_out/bench_dist.err
exit $rc
