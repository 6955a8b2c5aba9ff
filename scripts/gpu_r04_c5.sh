# Round 4: the whole C5 job emulated on one GPU (scripts/c5_full.py; a C2
# rehearsal of the same script first), the graph phase at C5 size
# (tests/test_gpu_scale.py::test_graph_phase_at_C5_size) and the host's CPU
# share as the CPU baseline sees it. Each step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04_c5
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())" > gpurun_out/r04_c5/cpu.txt
cat /sys/fs/cgroup/cpu.max >> gpurun_out/r04_c5/cpu.txt 2>&1 || true
cat gpurun_out/r04_c5/cpu.txt
timeout -k 10 300 python -u scripts/c5_full.py --config C2 --out gpurun_out/r04_c5/c2_full.json > gpurun_out/r04_c5/c2_full.log 2>&1
rc=$?; echo "C2 rehearsal rc=$rc"; tail -3 gpurun_out/r04_c5/c2_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -k graph_phase_at_C5 -x -v -s --timeout 380 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_c5/graph_test.log 2>&1
rc=$?; echo "graph test rc=$rc"; tail -3 gpurun_out/r04_c5/graph_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 780 python -u scripts/c5_full.py --config C5 --out gpurun_out/r04_c5/c5_full.json > gpurun_out/r04_c5/c5_full.log 2>&1
rc=$?; echo "C5 full rc=$rc"; tail -4 gpurun_out/r04_c5/c5_full.log
case $rc in 0|1) ;; *) exit $rc;; esac
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_c5/prof_C5s2 -o run -- python3 bench.py --config C5 --shard 2/8 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/r04_c5/prof_C5s2.log 2>&1
echo "C5 shard-2 rocprof rc=$?"
exit $rc
