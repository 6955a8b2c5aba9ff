# A/B runs of the quick bench under environment knobs (engine getenv):
# Usage: bash scripts/gpu_ab.sh "RC_ROW_WAVES=7" "RC_ROW_WAVES=8" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for kv in "" "$@"; do
  env $kv timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
  python scripts/ab_line.py gpurun_out/ab.json "$kv"
done
