# Rehearsal of bench.py's N > 1 path (frame sharding, barrier + max-over-ranks
# timing, error sum) on a one-GPU box: 2 and 4 ranks share the GPU over gloo.
# The numbers are not measurements (ranks contend for one GPU).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/rehearse_${1:-x}; mkdir -p $OUT
for N in 2 4; do
  OFDM_BENCH_SHARE_GPU=1 OFDM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --frames 40 \
    --steps 3 --warmup 1 --no-cpu > $OUT/n$N.json 2> $OUT/n$N.err
  rc=$?; echo "N=$N rc=$rc"; cat $OUT/n$N.json; [ $rc -eq 0 ] || exit $rc
done
