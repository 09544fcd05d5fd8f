#!/bin/bash
# round-2 profile set after the VALU / tile-start changes (configs[2]): GPU suite, bench line +
# summary, PMC passes (FETCH_SIZE / WRITE_SIZE / MFMA busy + wait shares), smoke
set -o pipefail
TAG=r02ay
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_$TAG.log 2>&1 || exit 1
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$PWD/gpurun_out/pmc_${TAG}_$i" -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-only > gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1
