#!/bin/bash
# PMC counter passes over the kernel microbenchmark (one rocprofv3 --pmc pass per counter group).
#   bash scripts/gpu_pmc_mb2.sh <tag> "<P D E>" "<counters pass 1>" ["<counters pass 2>" ...]
set -o pipefail
TAG=${1:-pmc}; shift
SHAPE=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$PWD/gpurun_out/pmcmb_${TAG}_$i" -o run \
    -- ./gnot-replication_amd/lib/microbench $SHAPE > gpurun_out/pmcmb_${TAG}_$i.log 2>&1 || exit 1
done
