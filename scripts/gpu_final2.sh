# Round-end refresh of the secondary evidence: full GPU suite, zero-forcing
# bench (defaults + A/B) with its rocprof stats, antenna-split bench (configs[4]
# slice, N=1).  usage: bash scripts/gpu_final2.sh <tag>
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}; OUT=gpurun_out/final_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
ZF_ARGS="--ab --U 16 4 8 32" bash scripts/gpu_zf.sh $TAG || exit 1
timeout -k 10 300 python -u bench.py --mode split --steps 10 --warmup 2 > $OUT/split.json 2> $OUT/split.err
rc=$?; echo "split rc=$rc"; cat $OUT/split.json; exit $rc
