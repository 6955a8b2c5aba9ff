# One timing-instrumented bench step (RC_ROW_TIMING build: seed-kernel phase
# cycles, row-kernel transition/step cycles) and a rocprofv3 kernel-stats pass.
# Usage: bash scripts/gpu_phase.sh [config]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=${1:-C3}
RC_LIB=rna_clique_amd/librcgpu_timing.so timeout -k 10 300 python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/phase_$CFG.json 2> gpurun_out/phase_$CFG.err
rc=$?; echo "timing rc=$rc"; grep "cycles" gpurun_out/phase_$CFG.err
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o run -- python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/prof_$CFG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(ls gpurun_out/prof_$CFG/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -25
exit $rc
