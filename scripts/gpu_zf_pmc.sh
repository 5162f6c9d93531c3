set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/zfpmc_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/zf_bench.py --ab --U 16 32 --no-cpu > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  for NT in 0 1; do
  i=$((i+1))
  OFDM_ZF_NT=$NT timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 scripts/zf_bench.py --U 16 --no-cpu --reps 2 --nsym 4000 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($P NT=$NT) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
