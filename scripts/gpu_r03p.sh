#!/bin/bash
# r03p: 32x32x16 chain-forward prototype vs the production chain2 forward (microbench), then r03o.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 gnot-replication_amd/lib/proto_c3 262144 5 20 > gpurun_out/r03p_proto.log 2>&1 || { cat gpurun_out/r03p_proto.log; exit 1; }
cat gpurun_out/r03p_proto.log
timeout -k 10 180 gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/r03p_mb.log 2>&1 || { cat gpurun_out/r03p_mb.log; exit 1; }
grep chain gpurun_out/r03p_mb.log
bash scripts/gpu_r03o.sh
