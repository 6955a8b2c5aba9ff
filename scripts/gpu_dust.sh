# DUST micro variants on random sequence and with 20 % poly-A tails.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for b in "$@"; do for pa in 0 0.2; do
  echo "== $b polyA=$pa"
  timeout -k 10 60 ./scratch/$b 1600000000 2560 $pa > gpurun_out/$b.txt 2>&1 || { cat gpurun_out/$b.txt; exit 1; }
  tail -3 gpurun_out/$b.txt
done; done
