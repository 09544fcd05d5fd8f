#!/bin/bash
# PMC traffic passes of the final round-3 tree: fp32 line and bf16 companion (FETCH_SIZE, WRITE_SIZE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--fp32-only" bash scripts/gpu_pmc.sh r03final_fp32 FETCH_SIZE WRITE_SIZE || exit 1
BENCH_ARGS="--dtype bf16" bash scripts/gpu_pmc.sh r03final_bf16 FETCH_SIZE WRITE_SIZE || exit 1
echo done
