# PMC passes (one counter group per run, kernel-trace only; no sys/hip tracing).
# Usage: bash scripts/gpu_pmc.sh [config] [groups...]; default: HBM bytes + instruction mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-C3}
shift || true
if [ $# -eq 0 ]; then
  set -- "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_$CFG/p$i -o run -- python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/pmc_${CFG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
