# DUST micro (random / 20 % poly-A tails, A/B phase cycles), then bench A/B of
# the DUST wave cap beside the new index sort on C3 and C3v.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for pa in 0 0.2; do
  echo "== dust polyA=$pa"
  timeout -k 10 60 ./scratch/dust_plain 1600000000 2560 $pa 2>&1 | tail -2 || exit 1
  timeout -k 10 60 ./scratch/dust_prof 1600000000 2560 $pa 2>&1 | tail -3 || exit 1
done
bash scripts/gpu_ab_env.sh C3 "RC_X=0" "RC_DUST_WAVES=2" "RC_DUST_WAVES=3" "RC_DUST_WAVES=4" "RC_SORT=rocprim" || exit 1
bash scripts/gpu_ab_env.sh C3v "RC_X=0" "RC_DUST_WAVES=3" "RC_DUST_WAVES=4"
