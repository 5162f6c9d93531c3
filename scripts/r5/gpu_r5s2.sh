set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 120 python -u scripts/r5/capture_debug.py
