# Round 4 (l): seed kernel at 6 workgroups per CU (128 subject samples per
# pass frees the LDS): 4 hits per lane (s6a) or 3 (s6b) against the default
# 5 per CU, C3 and C3v.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_l
mkdir -p $D
for cfg in C3 C3v; do
  reps=2; [ $cfg = C3v ] && reps=1
  for i in $(seq 1 $reps); do
    for v in base s6a s6b; do
      L=rna_clique_amd/librcgpu.so; [ $v != base ] && L=rna_clique_amd/librcgpu_$v.so
      RC_LIB=$L timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D/${cfg}_$v$i.json 2> $D/${cfg}_$v$i.err
      rc=$?; [ $rc -eq 0 ] || { echo "$cfg $v rc=$rc"; tail -5 $D/${cfg}_$v$i.err; exit $rc; }
      python3 -c "import json; d=json.load(open('$D/${cfg}_$v$i.json')); p=d['phases_ms']; print('$cfg $v', d['value'], d['ms_per_step'], p['seed_kernel_ms'], p['align_kernel_ms'], p['index_ms'])"
    done
  done
done
exit 0
