# Round 4 (y): the 8-rank C3 emulation (shared DUST) on the final sources.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${R04_TAG:-r04_y}
mkdir -p $D
timeout -k 10 400 python -u scripts/shard_time.py --config C3 --shards 8 --reps 2 --share-dust > $D/C3_shards8_sharedust.txt 2>&1
rc=$?; echo "shards rc=$rc"; grep -E "shard [0-9]" $D/C3_shards8_sharedust.txt; exit $rc
