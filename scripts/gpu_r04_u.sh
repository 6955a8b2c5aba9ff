# Round 4 (u): an HSP overflow redoes extend_kernel alone (not the row kernels;
# the buffer is first sized from the defer counts),
# alignment parity incl. the forced-retry test, the C3v config test
# (its first run overflows), and one-step C3v / C3 runs without warmup (the
# first run pays the retry) beside warm ones.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${R04_TAG:-r04_u}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/gpu_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $D/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "variant" -x -v --durations=0 --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep -E "passed|failed|s call" $D/gpu_configs.log | tail -4; [ $rc -eq 0 ] || exit $rc
for cfg in C3v C3; do
  for w in 0 1; do
    timeout -k 10 200 python bench.py --config $cfg --steps 1 --warmup $w --no-cpu-baseline --no-e2e > $D/${cfg}_w$w.json 2> $D/${cfg}_w$w.err
    rc=$?; [ $rc -eq 0 ] || { echo "$cfg w$w rc=$rc"; tail -5 $D/${cfg}_w$w.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$D/${cfg}_w$w.json')); p=d['phases_ms']; print('$cfg warmup $w', d['value'], d['ms_per_step'], 'ext', p['align_kernel_ms'], 'retries', p['ext_retries'])"
  done
done
exit 0
