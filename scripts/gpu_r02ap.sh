#!/bin/bash
# configs[1] after the size-based attention-pass choice (VALU below 512 chunks): bench A/B with the
# VALU state kernel, configs[2] unchanged check, GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --workload cfg2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ap_cfg2.json 2>gpurun_out/ap_cfg2.err &&
GNOT_STATE_VALU=1 timeout -k 10 300 python3 -u bench.py --workload cfg2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ap_cfg2_sv.json 2>/dev/null &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ap_cfg3.json 2>gpurun_out/ap_cfg3.err &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ap_tests.log 2>&1
