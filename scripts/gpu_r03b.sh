#!/bin/bash
# headline-size oracle parity (tests/test_gpu_headline.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_headline.py -m gpu -x -v -s --timeout 900 --timeout-method thread --durations=0 > gpurun_out/r03b_tests.log 2>&1
