# Round 4 final validation, part 2: the default bench line (C3, CPU baseline
# included), a rocprofv3 kernel-stats pass of the same command, and the PMC
# passes (one counter group per run, kernel trace only) for the roofline's
# traffic and the extension's issue rate.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${R04_TAG:-r04_final}
mkdir -p $D
nproc > $D/nproc.txt; lscpu > $D/lscpu.txt 2>&1 || true
timeout -k 10 600 python bench.py --config C3 --steps 10 --warmup 1 > $D/C3_bench.json 2> $D/C3_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 2500 $D/C3_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_C3 -o run -- python3 bench.py --config C3 --steps 3 --warmup 0 --no-cpu-baseline --no-e2e > $D/prof_C3.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $D/pmc_C3/p$i -o run -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $D/pmc_C3_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
