# Round 4 (t): job passes at C3v -- where the time goes. Kernel stats of one
# C3v step with jobs (RC_JOBS=1: 32-lane rows, 64-lane pass over the ones
# that outgrow the sub-band), without (RC_JOBS=0), and the jobs straight on
# 64-lane rows (RC_JOBS=2); bench lines of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${R04_TAG:-r04_t}
mkdir -p $D
for j in 2 1 0; do
  RC_JOBS=$j timeout -k 10 200 python bench.py --config C3v --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3v_j$j.json 2> $D/C3v_j$j.err
  rc=$?; [ $rc -eq 0 ] || { echo "C3v j$j rc=$rc"; tail -5 $D/C3v_j$j.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$D/C3v_j$j.json')); p=d['phases_ms']; print('C3v j$j', d['value'], d['ms_per_step'], 'ext', p['align_kernel_ms'], 'jobs', p['ext_jobs'], 'full', p['ext_fullband'], 'steps', p['ext_steps'])"
done
for j in 1 0 2; do
  RC_JOBS=$j timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_j$j -o run -- python3 bench.py --config C3v --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/prof_j$j.log 2>&1
  rc=$?; echo "prof j$j rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $D/prof_j$j -name "run_kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]: print('  %8.1f ms %4s %s' % (int(r['TotalDurationNs'])/1e6, r['Calls'], r['Name'][:70]))"
done
exit 0
