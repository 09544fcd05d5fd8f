#!/bin/bash
# scheduling knobs of the weight-gradient side stream at configs[2]: workgroup target (split-K) and
# side-stream priority
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 -u bench.py --steps 10 --warmup 3 --fp32-only --no-cpu-baseline"
timeout -k 10 240 $B > gpurun_out/ak_base.json 2>/dev/null &&
GNOT_WIDE_WGS=512 timeout -k 10 240 $B > gpurun_out/ak_wgs512.json 2>/dev/null &&
GNOT_WIDE_WGS=1280 timeout -k 10 240 $B > gpurun_out/ak_wgs1280.json 2>/dev/null &&
GNOT_SIDE_PRIO=1 timeout -k 10 240 $B > gpurun_out/ak_prio1.json 2>/dev/null &&
GNOT_SIDE_PRIO=-1 timeout -k 10 240 $B > gpurun_out/ak_prio-1.json 2>/dev/null
