set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do for w in 1 0; do C2D_ATTN_W8=$w TAG=w8=$w timeout -k 10 120 python -u scripts/attn_d40_check.py 2>&1 | grep "^w8" || exit 1; done; done
