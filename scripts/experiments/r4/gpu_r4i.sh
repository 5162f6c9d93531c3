# Round 4 session i: throughput of the staged any-C path (mixed-radix row FFT
# into the staging buffer + frequency-domain LS / MRC), R = 64, 400 frames,
# plus a kernel-trace profile of the C = 1536 run.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4i; mkdir -p $OUT
for C in 1536 600 1200 3000 6144 512 2048; do
  timeout -k 10 300 python bench.py --C $C --frames 400 --no-cpu --no-mode-a --steps 10 --warmup 3 \
    > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || { tail $OUT/bench_c$C.err; exit 1; }
  cut -c 1-300 $OUT/bench_c$C.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof1536 -o run -- python3 bench.py --C 1536 --frames 400 \
  --no-cpu --no-mode-a --steps 10 --warmup 3 > $OUT/prof1536.json 2> $OUT/prof1536.err || { tail $OUT/prof1536.err; exit 1; }
find $OUT/prof1536 -name "*kernel_stats.csv" -exec cat {} \; | cut -c 1-200
