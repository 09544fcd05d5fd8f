#!/bin/bash
# configs[1]: split-K workgroup target of the d=128 weight-gradient kernel (GNOT_X6_WGS), bench sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="timeout -k 10 200 python3 -u bench.py --workload cfg2 --no-cpu-baseline --steps 50 --warmup 10"
$B > gpurun_out/bb_256.json 2>/dev/null &&
GNOT_X6_WGS=128 $B > gpurun_out/bb_128.json 2>/dev/null &&
GNOT_X6_WGS=192 $B > gpurun_out/bb_192.json 2>/dev/null &&
GNOT_X6_WGS=384 $B > gpurun_out/bb_384.json 2>/dev/null &&
GNOT_X6_WGS=512 $B > gpurun_out/bb_512.json 2>/dev/null &&
GNOT_X6_WGS=64 $B > gpurun_out/bb_64.json 2>/dev/null &&
$B > gpurun_out/bb_256b.json 2>/dev/null
