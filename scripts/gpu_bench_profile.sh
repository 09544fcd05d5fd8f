#!/bin/bash
# Run on the GPU box (gpurun): bench line + rocprofv3 kernel-trace summary.
#   bash scripts/gpu_bench_profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-run}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --breakdown "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1
