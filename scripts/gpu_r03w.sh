#!/bin/bash
# r03w: smoke, the default bench line (fp32 + bf16 companion + cpu baseline), rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03w_smoke.log 2>&1 || { tail -20 gpurun_out/r03w_smoke.log; exit 1; }
tail -2 gpurun_out/r03w_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err || { tail -20 gpurun_out/r03w_bench.err; exit 1; }
cat gpurun_out/r03w_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_r03w" -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_r03w.log 2>&1 || { tail -20 gpurun_out/prof_r03w.log; exit 1; }
echo done
