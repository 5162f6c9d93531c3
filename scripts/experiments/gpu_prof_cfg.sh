#!/usr/bin/env bash
# Profile a non-default bench shape: bash scripts/experiments/gpu_prof_cfg.sh <tag> [bench args]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
TAG=$1; shift
bash scripts/gpu_profile.sh $TAG "$@" || { echo "profile failed"; exit 1; }
cd "$ROOT" && python scripts/pmc_summary.py gpurun_out/prof_$TAG $TAG notraffic | grep -E "^MRC|k_mrc|k_ls"
