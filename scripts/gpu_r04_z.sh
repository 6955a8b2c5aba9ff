# Round 4 (z): the driver's default bench command on the final sources, to
# confirm its line carries the committed PMC traffic (same src_hash).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${R04_TAG:-r04_z}
mkdir -p $D
timeout -k 10 600 python bench.py > $D/bench_default.json 2> $D/bench_default.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json; d=json.load(open('$D/bench_default.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:600])"; exit $rc
