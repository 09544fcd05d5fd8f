#!/bin/bash
# the other BASELINE workloads on the final tree, one GPU: configs[3]'s 1M-point mesh (MoE recompute
# chosen automatically), configs[4]'s 64 variable meshes (fixed and shuffled geometry), configs[1]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --workload cfg4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/an_cfg4.json 2> gpurun_out/an_cfg4.err &&
timeout -k 10 300 python3 -u bench.py --workload cfg5 --steps 10 --warmup 3 > gpurun_out/an_cfg5.json 2> gpurun_out/an_cfg5.err &&
timeout -k 10 300 python3 -u bench.py --workload cfg5 --steps 10 --warmup 3 --vary-geometry --no-cpu-baseline > gpurun_out/an_cfg5_vary.json 2> gpurun_out/an_cfg5_vary.err &&
timeout -k 10 300 python3 -u bench.py --workload cfg2 --steps 50 --warmup 10 > gpurun_out/an_cfg2.json 2> gpurun_out/an_cfg2.err
