# PMC HBM traffic of the default zero-forcing kernels (U=16 and U=32, 4000
# symbols): one FETCH_SIZE and one WRITE_SIZE pass each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/zfpmc2_${1:-x}; mkdir -p $OUT
i=0
for U in 16 32; do
  for P in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 scripts/zf_bench.py --U $U --no-cpu --reps 2 --nsym 4000 > $OUT/p$i.log 2>&1
    rc=$?; echo "pass $i (U=$U $P) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
