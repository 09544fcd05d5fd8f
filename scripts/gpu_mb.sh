#!/bin/bash
# GPU box: kernel microbenchmark at the given shapes.   bash scripts/gpu_mb.sh <tag> "<P D E>" ["<P D E>" ...]
set -o pipefail
TAG=${1:-mb}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for S in "$@"; do
  timeout -k 10 120 ./gnot-replication_amd/lib/microbench $S >> gpurun_out/mb_$TAG.txt 2>&1 || exit 1
done
