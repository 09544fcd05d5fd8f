#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 --pmc pass per counter group).
#   BENCH_ARGS="--fp32-only" bash scripts/gpu_pmc.sh <tag> "<counters pass 1>" "<counters pass 2>" ...
set -o pipefail
TAG=${1:-pmc}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$PWD/gpurun_out/pmc_${TAG}_$i" -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit 1
done
