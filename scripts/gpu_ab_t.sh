# A/B like gpu_ab.sh, plus one timing-instrumented bench step per value (needs a
# second library built with -DRC_ROW_TIMING at rna_clique_amd/librcgpu_timing.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VAR=$1; VALS=$2; CFG=${3:-C3}
bash scripts/gpu_ab.sh "$VAR" "$VALS" "$CFG" 3 || exit $?
if [ -f rna_clique_amd/librcgpu_timing.so ]; then
  for v in $VALS; do
    export $VAR=$v
    RC_LIB=rna_clique_amd/librcgpu_timing.so timeout -k 10 300 python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bt_$v.json 2> gpurun_out/bt_$v.err
    rc=$?; echo "[$VAR=$v] timing rc=$rc"; grep "wave-cycles" gpurun_out/bt_$v.err
    [ $rc -eq 0 ] || exit $rc
  done
fi
