#!/bin/bash
# r03wl: the GPU suite on the final round-3 tree, then the other BASELINE workloads (fp32, no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r03wl_tests.log 2>&1 || { tail -40 gpurun_out/r03wl_tests.log; exit 1; }
tail -1 gpurun_out/r03wl_tests.log
for w in cfg1 cfg2 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --fp32-only \
    > gpurun_out/r03wl_$w.json 2> gpurun_out/r03wl_$w.err || { tail -5 gpurun_out/r03wl_$w.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r03wl_$w.json
done
