# Round 4 (p): which per-CU resource bounds the seed kernel -- LDS (bank
# conflicts, issue waits), scalar memory, instruction cache, the issue mix.
# One counter group per run, kernel trace only, seed kernel launches only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_p
mkdir -p $D
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "seed_kernel|extend_rows" --output-format csv -d $D/pmc/p$i -o run -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/pmc_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/pmc_p$i.log; exit $rc; }
done
exit 0
