#!/bin/bash
# r03o: serial-stream kernel stats (true per-kernel cost without side-stream overlap) + PMC traffic passes
# for the fp32 headline and bf16 mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export GNOT_SERIAL_WGRAD=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_r03o_serial" -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_r03o_serial.log 2>&1 || exit 1
unset GNOT_SERIAL_WGRAD
BENCH_ARGS="--fp32-only" bash scripts/gpu_pmc.sh r03o_fp32 FETCH_SIZE WRITE_SIZE || exit 1
BENCH_ARGS="--dtype bf16" bash scripts/gpu_pmc.sh r03o_bf16 FETCH_SIZE WRITE_SIZE || exit 1
echo done
