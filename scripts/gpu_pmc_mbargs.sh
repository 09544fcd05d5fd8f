#!/bin/bash
# PMC counter passes over the kernel microbenchmark with arguments (one rocprofv3 --pmc pass per group).
#   bash scripts/gpu_pmc_mbargs.sh <tag> "<microbench args>" "<counters pass 1>" "<counters pass 2>" ...
set -o pipefail
TAG=${1:-mb}; ARGS=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
files=""
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$PWD/gpurun_out/pmcmb_${TAG}_$i" -o run \
    -- ./gnot-replication_amd/lib/microbench $ARGS > gpurun_out/pmcmb_${TAG}_$i.log 2>&1 || exit 1
  files="$files $(ls gpurun_out/pmcmb_${TAG}_$i/*counter_collection.csv gpurun_out/pmcmb_${TAG}_$i/*/*counter_collection.csv 2>/dev/null)"
done
python3 scripts/pmc_summary.py gpurun_out/pmcmb_${TAG}.csv $files
