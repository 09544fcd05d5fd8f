#!/bin/bash
# round-3 baseline: GPU suite, smoke, default bench line (after the wide-wgrad db-reduction barrier fix)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03a_smoke.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
