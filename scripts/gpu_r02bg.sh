#!/bin/bash
# forward pair mode in bf16 mode only (per-NP choice): GPU suite, smoke, default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/bg_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/bg_smoke.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/bg_bench.json 2> gpurun_out/bg_bench.err
