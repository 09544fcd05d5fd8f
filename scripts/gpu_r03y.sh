#!/bin/bash
# r03y: final-tree validation: the whole GPU suite, smoke, the default bench line, rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r03y_tests.log 2>&1 || { tail -40 gpurun_out/r03y_tests.log; exit 1; }
tail -2 gpurun_out/r03y_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y_smoke.log 2>&1 || { tail -20 gpurun_out/r03y_smoke.log; exit 1; }
tail -1 gpurun_out/r03y_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r03y_bench.json 2> gpurun_out/r03y_bench.err || { tail -20 gpurun_out/r03y_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03y_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac_pipe'], d['roofline']['traffic'], d['bf16_mode']['value'], d['bf16_mode']['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_r03y" -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_r03y.log 2>&1 || { tail -20 gpurun_out/prof_r03y.log; exit 1; }
echo done
