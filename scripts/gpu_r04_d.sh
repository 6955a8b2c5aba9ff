# Round 4 (d): split tiles' DUST over transcript ranges only (tile tests, C5
# rank-2 shard); what bounds the seed kernel, and the 8-rank C3 split.
#  1. random-line read rate of the chip (scripts/micro/rand_micro.hip)
#  2. 8 rank shards of C3 one after another (scripts/shard_time.py)
#  3. seed-kernel PMC passes (issue/wait mix, L2 hit/miss and fabric reads,
#     address-unit load), one pass per run, kernel-trace only
# Each step under its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r04_d
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "tiles or dust" > $D/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --shard 2/8 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/C5_shard2of8_bench.json 2> $D/C5_shard.err
rc=$?; echo "C5 shard rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/C5_shard.err; exit $rc; }
python3 -c "import json; d=json.load(open('$D/C5_shard2of8_bench.json')); p=d['phases_ms']; print('C5 s2', d['s_per_step'], {k: p[k] for k in ('index_ms','dust_ms','seed_kernel_ms','align_kernel_ms','index_reused','tiles')})"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -o $D/rand_micro scripts/micro/rand_micro.hip || exit 1
timeout -k 10 180 $D/rand_micro 16 64 > $D/rand_micro.txt 2>&1
rc=$?; echo "rand rc=$rc"; cat $D/rand_micro.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/shard_time.py --config C3 --shards 8 --reps 2 > $D/C3_shards8.txt 2>&1
rc=$?; echo "shards rc=$rc"; grep shard $D/C3_shards8.txt; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "seed_kernel|extend_rows" --output-format csv -d $D/pmc/p$i -o run -- python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/pmc_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $D/pmc_p$i.log; exit $rc; }
done
exit 0
