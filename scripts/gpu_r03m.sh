#!/bin/bash
# rehearsal of the driver's N>1 bench paths on the one-GPU box (2 ranks on cuda:0 over gloo, host-staged
# collectives): default N>1 workload configs[3] (one mesh point-sharded, reduced to 65,536 points so two
# ranks fit one GPU), the weak cfg3 path, sample-DP configs[4]; plus the RCCL point-shard step at world 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export GNOT_BENCH_BACKEND=gloo GNOT_BENCH_ONE_GPU=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 2 --steps 3 --warmup 2 --points 65536 > gpurun_out/r03m_n2_cfg4.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 \
  bench.py --gpus 2 --steps 3 --warmup 2 --workload cfg3 --points 32768 > gpurun_out/r03m_n2_cfg3.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 \
  bench.py --gpus 2 --steps 3 --warmup 2 --workload cfg5 --meshes 8 > gpurun_out/r03m_n2_cfg5.log 2>&1 &&
unset GNOT_BENCH_BACKEND GNOT_BENCH_ONE_GPU &&
GNOT_BENCH_FORCE_SHARD=1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --fp32-only > gpurun_out/r03m_force_shard.json 2> gpurun_out/r03m_force_shard.err
