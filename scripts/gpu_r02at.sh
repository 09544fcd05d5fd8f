#!/bin/bash
# no-SLP build + 13-VALU GELU + v_perm bf16 packing: microbench, GPU suite, configs[2] and configs[1]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/at_mb.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/at_tests.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/at_cfg3.json 2>/dev/null &&
timeout -k 10 300 python3 -u bench.py --workload cfg2 --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/at_cfg2.json 2>/dev/null
