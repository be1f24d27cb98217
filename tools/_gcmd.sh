set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in 1 2 3 4; do echo "matk=$k $(FBN_JT_VMATK=$k timeout -k 10 120 python tools/munin_once.py 125000 4 0 2>&1 | tail -1)" || exit 1; done
