# A/B of the bench only (no tests), once per value of an environment variable.
# Usage: bash scripts/gpu_ab_bench.sh VAR "v1 v2 ..." [config] [steps]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VAR=$1; VALS=$2; CFG=${3:-C3}; STEPS=${4:-3}
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 300 python bench.py --config "$CFG" --steps "$STEPS" --warmup 1 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err
  rc=$?; echo "[$VAR=$v] bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print(d['value'],d['ms_per_step']);print(d['phases_ms'])"
done
