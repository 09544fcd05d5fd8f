#!/bin/bash
# size-based attention-pass / state-kernel choice: every workload at defaults, cfg1/cfg5 A/B with the
# MFMA passes forced, GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline"
$B --workload cfg2 --steps 50 --warmup 10 > gpurun_out/aq_cfg2.json 2>gpurun_out/aq_cfg2.err &&
$B --workload cfg1 --steps 20 --warmup 5 > gpurun_out/aq_cfg1.json 2>gpurun_out/aq_cfg1.err &&
GNOT_APPLY_MFMA_MIN=0 GNOT_STATE_MFMA_MIN=0 $B --workload cfg1 --steps 20 --warmup 5 > gpurun_out/aq_cfg1_mfma.json 2>/dev/null &&
$B --workload cfg5 --steps 10 --warmup 3 > gpurun_out/aq_cfg5.json 2>gpurun_out/aq_cfg5.err &&
GNOT_APPLY_MFMA_MIN=0 GNOT_STATE_MFMA_MIN=0 $B --workload cfg5 --steps 10 --warmup 3 > gpurun_out/aq_cfg5_mfma.json 2>/dev/null &&
$B --steps 10 --warmup 3 > gpurun_out/aq_cfg3.json 2>gpurun_out/aq_cfg3.err &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/aq_tests.log 2>&1
