#!/bin/bash
# after the size-based attention choice: configs[2] A/B on one box (defaults vs MFMA forced), bench
# line with breakdown, kernel-trace summaries of configs[2] and configs[1], smoke
set -o pipefail
TAG=r02ar
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fp32-only"
$B --steps 10 --warmup 3 > gpurun_out/${TAG}_cfg3_a.json 2>/dev/null || exit 1
GNOT_APPLY_MFMA_MIN=0 GNOT_STATE_MFMA_MIN=0 $B --steps 10 --warmup 3 > gpurun_out/${TAG}_cfg3_mfma.json 2>/dev/null || exit 1
$B --steps 10 --warmup 3 > gpurun_out/${TAG}_cfg3_b.json 2>/dev/null || exit 1
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_cfg3" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_${TAG}_cfg3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_cfg2" -o run --output-format csv \
  -- python3 bench.py --workload cfg2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}_cfg2.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1
