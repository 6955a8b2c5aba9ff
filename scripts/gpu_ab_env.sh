# Bench lines (no CPU baseline, no e2e leg) for one config under several
# environment settings. Usage: bash scripts/gpu_ab_env.sh CONFIG "K=V" "K=V" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=$1; shift
for kv in "$@"; do
  env $kv timeout -k 10 400 python bench.py --config "$CFG" --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab_$CFG.json 2> gpurun_out/ab_$CFG.err || exit $?
  python scripts/ab_line.py gpurun_out/ab_$CFG.json "$CFG $kv"
done
