# Round 4 (s): job passes -- the later seeds of multi-HSP searches on the row
# kernels instead of extend_kernel: alignment parity, the C3 / C3v config
# tests (20 oracle pairs covering every sample), then C3 / C3v A/B: jobs
# (default) vs RC_JOBS=0, and the 8-waves-per-SIMD row kernel (librcgpu_w8.so,
# the previous sources).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${R04_TAG:-r04_s}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/gpu_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $D/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "C3" -x -v --durations=0 --timeout 400 --timeout-method thread -p no:cacheprovider > $D/gpu_configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep -E "passed|failed|s call" $D/gpu_configs.log | tail -6; [ $rc -eq 0 ] || exit $rc
run() {  # cfg tag lib env...
  cfg=$1; tag=$2; L=$3; shift 3
  env RC_LIB=$L "$@" timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D/${cfg}_$tag.json 2> $D/${cfg}_$tag.err
  rc=$?; [ $rc -eq 0 ] || { echo "$cfg $tag rc=$rc"; tail -5 $D/${cfg}_$tag.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$D/${cfg}_$tag.json')); p=d['phases_ms']; print('$cfg $tag', d['value'], d['ms_per_step'], 'seed', p['seed_kernel_ms'], 'ext', p['align_kernel_ms'], 'idx', p['index_ms'], 'jobs', p.get('ext_jobs'), 'left', p.get('defer_left'), 'defer', p.get('ext_deferred'))"
}
M=rna_clique_amd/librcgpu.so; W8=rna_clique_amd/librcgpu_w8.so
run C3v jobs $M RC_JOBS=1
run C3v nojobs $M RC_JOBS=0
run C3 jobs1 $M RC_JOBS=1
run C3 w8a $W8 RC_JOBS=1
run C3 jobs2 $M RC_JOBS=1
run C3 w8b $W8 RC_JOBS=1
run C3v w8 $W8 RC_JOBS=0
exit 0
