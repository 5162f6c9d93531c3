# Round-end refresh: GPU tests, headline profile (+PMC) and bench, then the
# C=4096 cfg5-slice profile.  usage: bash scripts/gpu_final.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${1:-r1e}
bash scripts/gpu_round.sh $TAG || exit $?
cd "$ROOT"
bash scripts/gpu_profile.sh c4kh --R 32 --C 4096 --frames 400 || { echo "c4k profile failed"; exit 1; }
cd "$ROOT"
python scripts/pmc_summary.py gpurun_out/prof_c4kh c4kh notraffic > /dev/null || exit 1
mkdir -p gpurun_out/profiles_c4kh && cp profiles/c4kh_* gpurun_out/profiles_c4kh/
echo "c4kh done"; tail -3 profiles/c4kh_summary.md
