#!/bin/bash
# configs[1] (d=128) step profile: kernel trace of the bench, and the same with the VALU attention
# passes (GNOT_APPLY_VALU / GNOT_STATE_VALU) for A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_ao" -o run --output-format csv \
  -- python3 bench.py --workload cfg2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_ao.log 2>&1 &&
GNOT_APPLY_VALU=1 GNOT_STATE_VALU=1 timeout -k 10 300 python3 -u bench.py --workload cfg2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ao_cfg2_valu.json 2>/dev/null &&
timeout -k 10 300 python3 -u bench.py --workload cfg2 --steps 50 --warmup 10 --no-cpu-baseline --no-graph > gpurun_out/ao_cfg2_eager.json 2>/dev/null
