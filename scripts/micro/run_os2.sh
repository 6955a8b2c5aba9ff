set -o pipefail
cd "$GRAFT_REPO_ROOT"
for b in "$@"; do echo "== $b"; timeout -k 10 120 ./scratch/$b || exit 1; done
