#!/bin/bash
# configs[2]: split-K workgroup target of the wide weight-gradient kernel (GNOT_WIDE_WGS) re-swept on
# the final kernels (fp32 line only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --fp32-only --steps 8 --warmup 3"
$B > gpurun_out/bh_256.json 2>/dev/null &&
GNOT_WIDE_WGS=192 $B > gpurun_out/bh_192.json 2>/dev/null &&
GNOT_WIDE_WGS=320 $B > gpurun_out/bh_320.json 2>/dev/null &&
GNOT_WIDE_WGS=384 $B > gpurun_out/bh_384.json 2>/dev/null &&
GNOT_WIDE_WGS=512 $B > gpurun_out/bh_512.json 2>/dev/null &&
$B > gpurun_out/bh_256b.json 2>/dev/null
