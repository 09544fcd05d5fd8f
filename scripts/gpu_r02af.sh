#!/bin/bash
# chain2 backward: writes gelu(h) in place; weight gradients read it as is; microbench, GPU suite, bench,
# rocprof kernel trace, smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/af_mb.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/af_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/af_bench.json 2> gpurun_out/af_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_af" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_af.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/af_smoke.log 2>&1
