#!/bin/bash
# generic widths: parity of d in {16, 80, 96, 112, 144, 160, 192} x head widths {4, 12, 16, 20, 24, 28, 32, 48}
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_widths.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r03k_widths.log 2>&1
