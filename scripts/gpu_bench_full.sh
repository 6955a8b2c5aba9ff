# The driver's bench command (defaults) and the rocprofv3 kernel stats of a
# 2-step run, then the PMC passes of one step. Usage: bash scripts/gpu_bench_full.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof.sh C3 $TAG || exit $?
bash scripts/gpu_pmc.sh C3 "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
