# Timing-only variants of the onesweep pass (no look-back / no stores): where a pass's time goes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OS_COPY=1 OS_ONLY_BIG=1 timeout -k 10 120 ./scratch/os_base || exit 1
for b in os_nolb os_nost os_nolbst; do echo "== $b"; OS_ONLY_BIG=1 timeout -k 10 120 ./scratch/$b; done
exit 0
