# split mode chunk size: 50 / 100 / 200 frames per chunk (one box, same session)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5w
for ch in 50 100 200 50; do
  timeout -k 10 300 python -u bench.py --mode split --no-cpu --chunk $ch > gpurun_out/r5w/split_c$ch.json 2> gpurun_out/r5w/split.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5w/split_c$ch.json').read().strip().splitlines()[-1]); print($ch, round(d['ms_per_step'],3), round(d['value']/1e6,3), {k: round(v,3) for k,v in d['stages_ms'].items() if isinstance(v,float)})"
done
