# Round 4 (e): where the seed kernel's block-cycles go (RC_ROW_TIMING build,
# librcgpu_timing.so) at C3 and on one C3 rank of eight, and the row kernel's
# instruction mix (one PMC pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_e
mkdir -p $D
RC_LIB=rna_clique_amd/librcgpu_timing.so timeout -k 10 200 python bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_timing.json 2> $D/C3_timing.err
rc=$?; echo "C3 timing rc=$rc"; grep -a "block-cycles\|wave-cycles" $D/C3_timing.err; [ $rc -eq 0 ] || exit $rc
RC_LIB=rna_clique_amd/librcgpu_timing.so timeout -k 10 200 python bench.py --config C3 --shard 4/8 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $D/C3_r4_timing.json 2> $D/C3_r4_timing.err
rc=$?; echo "C3 rank-4 timing rc=$rc"; grep -a "block-cycles\|wave-cycles" $D/C3_r4_timing.err; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "seed_kernel|extend_rows|dust_kernel|onesweep|kmer_fill" --output-format csv -d $D/pmc/p1 -o run -- python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/pmc_p1.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
