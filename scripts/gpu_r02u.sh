#!/bin/bash
# default bench line (fp32 headline + companion bf16 measurement + CPU baseline), its rocprof kernel
# trace (fp32 only), smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/u_bench.json 2> gpurun_out/u_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_u" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_u.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/u_smoke.log 2>&1
