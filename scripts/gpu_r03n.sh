#!/bin/bash
# overlap A/B: weight gradients on the side stream (default) vs serial on the main stream, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --breakdown > gpurun_out/r03n_overlap_$i.json 2> gpurun_out/r03n_overlap_$i.err || exit 1
  GNOT_SERIAL_WGRAD=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --breakdown > gpurun_out/r03n_serial_$i.json 2> gpurun_out/r03n_serial_$i.err || exit 1
done
