# Round 4 (v): the reverse pass runs only the genes with a near-mask hit
# (rev_filter_kernel): alignment parity (reverse-only seeds asserted), the C3
# and C3v config tests, and C3 / C3v A/B against RC_REV_FILTER=0.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${R04_TAG:-r04_v}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/gpu_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $D/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
run() {  # cfg tag env...
  cfg=$1; tag=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D/${cfg}_$tag.json 2> $D/${cfg}_$tag.err
  rc=$?; [ $rc -eq 0 ] || { echo "$cfg $tag rc=$rc"; tail -5 $D/${cfg}_$tag.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$D/${cfg}_$tag.json')); p=d['phases_ms']; print('$cfg $tag', d['value'], d['ms_per_step'], 'seed', p['seed_kernel_ms'], 'ext', p['align_kernel_ms'], 'idx', p['index_ms'], 'rs', p['reverse_seeds'])"
}
run C3 filt1 RC_REV_FILTER=1
run C3 nofilt1 RC_REV_FILTER=0
run C3 filt2 RC_REV_FILTER=1
run C3 nofilt2 RC_REV_FILTER=0
run C3v filt RC_REV_FILTER=1
run C3v nofilt RC_REV_FILTER=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "C3" -x -v --durations=0 --timeout 400 --timeout-method thread -p no:cacheprovider > $D/gpu_configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep -E "passed|failed|s call" $D/gpu_configs.log | tail -4; exit $rc
