# round 6 (o): stamps of the split-estimator build at configs[1] (estimator phases, workgroup timeline)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6o; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --R 16 --frames 100 --steps 200 --warmup 50 --no-cpu --stamps-out $OUT/stamps_cfg1.npy > $OUT/cfg1.json 2> $OUT/cfg1.err || { tail $OUT/cfg1.err; exit 1; }
python3 scripts/est_phases.py $OUT/stamps_cfg1.npy 200 > $OUT/phases.txt && cat $OUT/phases.txt
python3 scripts/wg_timeline.py $OUT/stamps_cfg1.npy --nls 200 > $OUT/timeline.txt && cat $OUT/timeline.txt
