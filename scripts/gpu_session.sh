#!/usr/bin/env bash
# One GPU session of named steps, each under its own time limit, stopping at
# the first failure (no retries).  Outputs under gpurun_out/<tag>/.
# usage: bash scripts/gpu_session.sh <tag> step [step ...]
# steps:
#   suite      pytest -m gpu (the driver's form)          smoke    __graft_entry__.smoke()
#   default    bench.py (driver form: 20 steps, 3 warm-up, CPU baseline) + stamps
#   cfg1       configs[1]: --R 16 --frames 100 --steps 20 --warmup 5 + stamps
#   cfg1_200   configs[1] at a steady clock: 200 steps after 50 warm-up steps
#   cfg2       configs[2]: --R 64 --C 2048 --frames 1000 --steps 10
#   c4096      configs[4] per-GPU slice: --R 32 --C 4096 --frames 400 --steps 20 + stamps
#   split      bench.py --mode split (RCCL, world 1) with stages_ms
#   freq       bench.py --mode freq (mode A line)
#   prof_default / prof_cfg1 / prof_c4096   scripts/gpu_prof_r4.sh of that command
#   clk_cfg1 / clk_default   scripts/dispatch_clock.py: per-dispatch clock + timeline (diagnostic build)
#   abx:<args> python scripts/abx.py <args, ':' for spaces>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
bench() { name=$1; lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; tail -c 3000 $OUT/$name.json; return $rc; }
for st in "$@"; do
  case $st in
    suite) timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
           rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
           rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log ;;
    default) bench default 600 --gpus 1 --steps 20 --warmup 5 --stamps-out $OUT/stamps_default.npy; rc=$? ;;
    cfg1) bench cfg1 300 --R 16 --frames 100 --steps 20 --warmup 5 --no-cpu --stamps-out $OUT/stamps_cfg1.npy; rc=$? ;;
    cfg1_200) bench cfg1_200 300 --R 16 --frames 100 --steps 200 --warmup 50 --no-cpu; rc=$? ;;
    cfg2) bench cfg2 300 --R 64 --C 2048 --frames 1000 --steps 10 --no-cpu --stamps-out $OUT/stamps_cfg2.npy; rc=$? ;;
    c4096) bench c4096 300 --R 32 --C 4096 --frames 400 --steps 20 --no-cpu --stamps-out $OUT/stamps_c4096.npy; rc=$? ;;
    split) bench split 300 --mode split --no-cpu; rc=$? ;;
    freq) bench freq 300 --mode freq --no-cpu; rc=$? ;;
    prof_default) timeout -k 10 1000 bash scripts/gpu_prof_r4.sh ${TAG}_default > $OUT/prof_default.log 2>&1; rc=$?; echo "prof_default rc=$rc"; tail -3 $OUT/prof_default.log ;;
    prof_cfg1) timeout -k 10 600 bash scripts/gpu_prof_r4.sh ${TAG}_cfg1 --gpus 1 --steps 20 --warmup 5 --R 16 --frames 100 > $OUT/prof_cfg1.log 2>&1; rc=$?; echo "prof_cfg1 rc=$rc"; tail -3 $OUT/prof_cfg1.log ;;
    prof_c4096) timeout -k 10 800 bash scripts/gpu_prof_r4.sh ${TAG}_c4096 --gpus 1 --steps 20 --warmup 5 --R 32 --C 4096 --frames 400 > $OUT/prof_c4096.log 2>&1; rc=$?; echo "prof_c4096 rc=$rc"; tail -3 $OUT/prof_c4096.log ;;
    clk_cfg1) for g in 0 9; do timeout -k 10 200 python -u scripts/dispatch_clock.py --R 16 --frames 100 --steps 20 --warmup 5 --gap-ms $g --tag cfg1_gap$g >> $OUT/clk_cfg1.jsonl 2>> $OUT/clk.err || { rc=1; break; }; done
              timeout -k 10 200 python -u scripts/dispatch_clock.py --R 16 --frames 100 --steps 200 --warmup 5 --tag cfg1_200 >> $OUT/clk_cfg1.jsonl 2>> $OUT/clk.err; rc=$?
              echo "clk_cfg1 rc=$rc"; grep summary $OUT/clk_cfg1.jsonl ;;
    clk_default) timeout -k 10 300 python -u scripts/dispatch_clock.py --R 64 --frames 1250 --steps 20 --warmup 5 --gap-ms 9 --tag default >> $OUT/clk_default.jsonl 2>> $OUT/clk.err; rc=$?
              echo "clk_default rc=$rc"; grep summary $OUT/clk_default.jsonl ;;
    prof_split) timeout -k 10 800 bash scripts/gpu_prof_r4.sh ${TAG}_split --gpus 1 --steps 20 --warmup 5 --mode split > $OUT/prof_split.log 2>&1; rc=$?; echo "prof_split rc=$rc"; tail -3 $OUT/prof_split.log ;;
    abx:*) a=${st#abx:}; timeout -k 10 600 python -u scripts/abx.py ${a//:/ } > $OUT/abx_$(echo $a | tr -c 'a-zA-Z0-9' _).jsonl 2> $OUT/abx.err; rc=$?; echo "abx $a rc=$rc"; tail -8 $OUT/abx_$(echo $a | tr -c 'a-zA-Z0-9' _).jsonl ;;
    *) echo "unknown step $st"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || exit $rc
done
echo "session $TAG done"
