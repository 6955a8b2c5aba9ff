# Round 4 (h): where the seed kernel's block-cycles go, finer (prologue,
# usability, lookup, hit loads / pre-test / full test; RC_ROW_TIMING build),
# then the whole C5s job on this one GPU (8 rank shards one after another,
# their edges into a graph-only engine, the matrix and its checks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_h
mkdir -p $D
RC_LIB=rna_clique_amd/librcgpu_timing.so timeout -k 10 200 python bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_timing.json 2> $D/C3_timing.err
rc=$?; echo "C3 timing rc=$rc"; grep -a "block-cycles" $D/C3_timing.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u scripts/c5_full.py --config C5s --out $D/c5s_full.json > $D/c5s_full.log 2>&1
rc=$?; echo "C5s full rc=$rc"; tail -4 $D/c5s_full.log
exit $rc
