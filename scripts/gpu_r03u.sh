#!/bin/bash
# r03u: chain backward weight ring (3 chunks in flight; h DMA ordered before the weight DMA): microbench, then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 150 gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/r03u_mb.log 2>&1 || { cat gpurun_out/r03u_mb.log; exit 1; }
grep chain gpurun_out/r03u_mb.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r03u_tests.log 2>&1 || { tail -40 gpurun_out/r03u_tests.log; exit 1; }
tail -3 gpurun_out/r03u_tests.log
