# round 6 (w): receiver phases of the one-launch demod (diagnostic build stamps) at configs[1] and the headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6w; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --R 16 --frames 100 --steps 200 --warmup 50 --no-cpu --stamps-out $OUT/stamps_cfg1.npy > $OUT/cfg1.json 2> $OUT/cfg1.err || { tail $OUT/cfg1.err; exit 1; }
python3 scripts/rx_phases.py $OUT/stamps_cfg1.npy 104 > $OUT/rx_cfg1.txt && cat $OUT/rx_cfg1.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --stamps-out $OUT/stamps_head.npy > $OUT/head.json 2> $OUT/head.err || { tail $OUT/head.err; exit 1; }
python3 scripts/rx_phases.py $OUT/stamps_head.npy 1256 > $OUT/rx_head.txt && cat $OUT/rx_head.txt
