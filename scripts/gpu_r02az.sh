#!/bin/bash
# weight-gradient row loads with the nt cache policy (microbench_prev / libprev.so, GNOT_WGRAD_AUX=2)
# vs default: interleaved microbench and configs[2] bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gnot-replication_amd/lib
timeout -k 10 200 ./$L/microbench_prev 262144 256 8 > gpurun_out/az_mb_nt_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/az_mb_1.txt 2>&1 &&
GNOT_LIB=$PWD/$L/libprev.so timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fp32-only --steps 10 --warmup 3 > gpurun_out/az_cfg3_nt.json 2>/dev/null &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fp32-only --steps 10 --warmup 3 > gpurun_out/az_cfg3.json 2>/dev/null &&
GNOT_LIB=$PWD/$L/libprev.so timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fp32-only --steps 10 --warmup 3 > gpurun_out/az_cfg3_nt_2.json 2>/dev/null &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fp32-only --steps 10 --warmup 3 > gpurun_out/az_cfg3_2.json 2>/dev/null
