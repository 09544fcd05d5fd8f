#!/bin/bash
# bf16 mode: bench line with the bf16-row weight-gradient class, rocprof kernel stats of the bf16 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --dtype bf16 --breakdown > gpurun_out/r03j_bf16_bench.json 2> gpurun_out/r03j_bf16_bench.err &&
export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r03j_bf16" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype bf16 > gpurun_out/prof_r03j_bf16.log 2>&1
