#!/bin/bash
# r03wl: the other BASELINE workloads on the final round-3 tree (fp32, no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in cfg1 cfg2 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --fp32-only \
    > gpurun_out/r03wl_$w.json 2> gpurun_out/r03wl_$w.err || { tail -5 gpurun_out/r03wl_$w.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r03wl_$w.json
done
