# One parameterised GPU-box script (run through gpurun): every step writes
# under gpurun_out/$TAG/ and appends the exact command it ran to
# gpurun_out/$TAG/commands.txt, so each profiles/<tag>/ says what produced it.
#
#   bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Steps (each under its own time limit; the script stops at the first failure):
#   smoke            __graft_entry__.smoke()
#   tests            every -m gpu test, one process
#   tests:EXPR       -m gpu tests matching -k EXPR
#   bench[:CFG]      bench.py --config CFG (default C3), 3 steps, no CPU baseline, no e2e
#   benchfull        bench.py with its defaults (CPU baseline + wall-clock leg)
#   e2e[:CFG]        bench.py with the wall-clock leg, no CPU baseline
#   stats[:CFG]      rocprofv3 --kernel-trace --stats of bench.py --config CFG
#   pmc[:CFG]        the PMC passes of scripts/gpu_pmc.sh (same-source counters)
#   pmcx:CFG:G1;G2   PMC passes with the given counter groups (';' between passes,
#                    ',' between counters), one rocprofv3 run each
#   counters         rocprofv3 -L (the counters this box's agent has)
#   shard:CFG:R/S    bench.py --shard R/S --config CFG (1 step, 1 warmup)
#   shardprof:CFG:R/S  the same under rocprofv3 --kernel-trace --hip-trace --stats
#   c5full[:CFG]     scripts/c5_full.py (default C5s)
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (ARGS: commas become spaces)
#   bin:NAME[:ARGS]  benchbin/NAME ARGS (a micro-benchmark built here, in-tree)
#   pmcbin:NAME:ARGS the same under one rocprofv3 PMC pass (instruction mix and waits)
#   env:VAR=VALUE    export VAR=VALUE for the later steps (A/B knobs); output
#                    names of later bench/stats steps carry _VAR=VALUE
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
ET=""
D=gpurun_out/$TAG
mkdir -p "$D"
log() { echo "$*" >> "$D/commands.txt"; }
run() {   # run LIMIT OUTFILE CMD...: one GPU step under its own time limit
  local lim=$1 out=$2; shift 2
  log "timeout -k 10 $lim $* > $out 2>&1"
  timeout -k 10 "$lim" "$@" > "$out" 2>&1
  local rc=$?
  echo "[$TAG] $* -> rc=$rc"; tail -3 "$out"
  return $rc
}
for step in "$@"; do
  IFS=: read -r kind a b <<< "$step"
  case $kind in
    smoke) run 300 "$D/smoke.log" python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    tests) if [ -n "$a" ]; then
             run 1100 "$D/gpu_tests_$a.log" python -u -m pytest tests -m gpu -k "$a" -x -v --timeout 700 --timeout-method thread -p no:cacheprovider || exit $?
           else
             run 1100 "$D/gpu_tests.log" python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread -p no:cacheprovider || exit $?
           fi ;;
    env) export "$a"; ET="${ET}_${a//\//_}"; log "export $a" ;;
    bench) c=${a:-C3}; run 600 "$D/${c}_bench${ET}.json" python bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e || exit $? ;;
    benchfull) run 900 "$D/bench_default.json" python bench.py || exit $? ;;
    e2e) c=${a:-C3}; run 600 "$D/${c}_e2e.json" python bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline || exit $? ;;
    stats) c=${a:-C3}
           run 600 "$D/${c}_stats${ET}.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$D/${c}_stats${ET}" -o run -- python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e || exit $? ;;
    pmc) c=${a:-C3}; log "bash scripts/gpu_pmc.sh $c  (-> gpurun_out/pmc_$c)"; bash scripts/gpu_pmc.sh "$c" || exit $? ;;
    pmcx) IFS=';' read -ra groups <<< "$b"; i=0
          for grp in "${groups[@]}"; do
            i=$((i+1))
            run 300 "$D/pmcx_${a}_p$i.log" rocprofv3 --kernel-trace --pmc ${grp//,/ } --output-format csv -d "$D/pmcx_$a/p$i" -o run -- python3 bench.py --config "$a" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e || exit $?
          done ;;
    counters) run 120 "$D/counters.txt" rocprofv3 -L || exit $? ;;
    shard) run 900 "$D/${a}_shard${b//\//of}${ET}.json" python -u bench.py --shard "$b" --config "$a" --steps 1 --warmup 1 || exit $? ;;
    shardprof) P="$D/${a}_shardprof${b//\//of}"
           run 900 "$P.log" rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d "$P" -o run -- python3 -u bench.py --shard "$b" --config "$a" --steps 1 --warmup 1 || exit $?
           T=$(python3 -c "import json,sys; print(int([json.loads(l) for l in open('$P.log') if l.startswith('{\"metric')][-1]['phases_ms']['tiles']))")
           log "python3 scripts/trace_gaps.py $P $T $P.gaps.json"
           python3 scripts/trace_gaps.py "$P" "$T" "$P.gaps.json" > /dev/null; rc=$?
           find "$P" \( -name '*_trace.csv' -o -name '*.db' \) -delete   # (hundreds of MB; the summaries stay)
           [ $rc -eq 0 ] || exit $rc ;;
    c5full) c=${a:-C5s}; run 1100 "$D/${c}_full.log" python -u scripts/c5_full.py --config "$c" --outputs /tmp/rc_c5_outputs --out "$D/${c}_full.json" || exit $? ;;
    bin) run 300 "$D/${a}_${b//,/_}.log" "benchbin/$a" ${b//,/ } || exit $? ;;
    pmcbin) run 300 "$D/pmc_${a}.log" rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d "$D/pmc_$a" -o run -- "benchbin/$a" ${b//,/ } || exit $? ;;
    py) run 900 "$D/$(basename "$a" .py).log" python -u "$a" ${b//,/ } || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
