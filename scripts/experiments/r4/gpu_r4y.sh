# Round 4 session y: GPU suite after the exact-twiddle changes (6144 receiver,
# generic stages), and bench lines at 6144, 1200 and 1536.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in 6144 1200 1536; do
  F=400; [ $C = 6144 ] && F=100
  timeout -k 10 300 python bench.py --C $C --frames $F --no-cpu --no-mode-a --steps 10 --warmup 3 \
    > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || { tail $OUT/bench_c$C.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c$C.json').read().strip().splitlines()[-1]); print($C, round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['frac'],3), d['check']['qpsk_symbol_errors'])"
done
