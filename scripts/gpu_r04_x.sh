# Round 4 (x): bench lines of the other configurations on the final sources
# (C1, C2, C3v, C4; C3 is r04_final3's), warm steps, no CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${R04_TAG:-r04_x}
mkdir -p $D
for cfg in C1 C2 C3v C4; do
  st=3; [ $cfg = C1 ] && st=10
  timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline --no-e2e > $D/${cfg}_bench.json 2> $D/${cfg}_bench.err
  rc=$?; [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; tail -5 $D/${cfg}_bench.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$D/${cfg}_bench.json')); p=d['phases_ms']; print('$cfg', d['value'], d['unit'], d['ms_per_step'], 'seed', p['seed_kernel_ms'], 'ext', p['align_kernel_ms'], 'idx', p['index_ms'])"
done
exit 0
