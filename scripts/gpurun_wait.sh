# Run one gpurun command, retrying ONLY while the pool has no free box
# (gpurun exit 3: nothing ran, nothing charged). Any other exit ends it.
# Usage: bash scripts/gpurun_wait.sh TIMEOUT_S LOGFILE 'command'
T=$1; LOG=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -eq 3 ] || break
  echo "no free box (try $i), waiting" >> "$LOG.wait"
  sleep 150
done
echo "exit $rc" >> "$LOG"
exit $rc
