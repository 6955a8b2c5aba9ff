# Round 4 (n): the current sources at scale -- the 8-rank C3 shard times with
# shared DUST masks (refitted planner, 5-workgroup seed kernel), a C3v kernel
# profile, then the whole C5s job again on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_n
mkdir -p $D
timeout -k 10 400 python -u scripts/shard_time.py --config C3 --shards 8 --reps 2 --share-dust > $D/C3_shards8_sharedust.txt 2>&1
rc=$?; echo "shards rc=$rc"; grep shard $D/C3_shards8_sharedust.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_C3v -o run -- python3 bench.py --config C3v --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/prof_C3v.log 2>&1
rc=$?; echo "rocprof C3v rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u scripts/c5_full.py --config C5s --out $D/c5s_full.json > $D/c5s_full.log 2>&1
rc=$?; echo "C5s full rc=$rc"; tail -3 $D/c5s_full.log
exit $rc
