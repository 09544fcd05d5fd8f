#!/bin/bash
# configs[2] profile set: bench line + breakdown, rocprofv3 kernel-trace summary, PMC passes
# (FETCH_SIZE / WRITE_SIZE / SQ busy+MFMA counters), each pass its own run.
set -o pipefail
TAG=${1:-r02k}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit 1
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$PWD/gpurun_out/pmc_${TAG}_$i" -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit 1
done
