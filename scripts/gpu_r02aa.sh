#!/bin/bash
# RCCL shard path (world-1 test + forced-shard bench at configs[2]), rocprof kernel trace of the default
# bench, smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread > gpurun_out/aa_shard.log 2>&1 &&
GNOT_BENCH_FORCE_SHARD=1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --fp32-only --no-cpu-baseline --breakdown > gpurun_out/aa_bench_shard1.json 2> gpurun_out/aa_bench_shard1.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_aa" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_aa.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/aa_smoke.log 2>&1
