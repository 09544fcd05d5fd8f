#!/bin/bash
# round-3: full GPU suite on the tree with bf16 storage, input grads, grid default, smoke, default bench line, rocprof kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03i_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03i_smoke.log 2>&1 &&
timeout -k 10 500 python3 -u bench.py --breakdown > gpurun_out/r03i_bench.json 2> gpurun_out/r03i_bench.err &&
export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r03i" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_r03i.log 2>&1
