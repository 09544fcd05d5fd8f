#!/bin/bash
# A/B: the library built without SLP vectorization (-fno-slp-vectorize: no packed f32 VALU beside the
# MFMAs) vs the default build; microbench twice each, interleaved, then the configs[2] bench both ways
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gnot-replication_amd/lib
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/as_mb_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench_noslp 262144 256 8 > gpurun_out/as_mb_noslp_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/as_mb_2.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench_noslp 262144 256 8 > gpurun_out/as_mb_noslp_2.txt 2>&1 &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/as_cfg3.json 2>/dev/null &&
GNOT_LIB=$PWD/$L/libgnot_hip_noslp.so timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/as_cfg3_noslp.json 2>/dev/null
