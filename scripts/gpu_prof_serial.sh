#!/bin/bash
# rocprofv3 kernel stats of a short bench run with the weight-gradient side stream disabled
# (uncontended per-kernel durations).   bash scripts/gpu_prof_serial.sh <tag>
set -o pipefail
TAG=${1:-serial}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_$TAG" -o run \
  --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
