#!/bin/bash
# microbench only (wide-wgrad diagnostics: no-GELU / L2-resident rows)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/ad_mb.txt 2>&1
