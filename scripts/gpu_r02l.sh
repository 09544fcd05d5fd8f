#!/bin/bash
# side2 fork/join fix (graph capture in the default bench), GPU suite, per-step geometry change cost
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/l_bench.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/l_tests.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --workload cfg5 --meshes 16 --no-graph --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/l_cfg5_fixed.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --workload cfg5 --meshes 16 --vary-geometry --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/l_cfg5_vary.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --workload cfg5 --meshes 16 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/l_cfg5_graph.log 2>&1
