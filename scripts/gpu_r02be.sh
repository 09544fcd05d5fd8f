#!/bin/bash
# final-tree rehearsal of the N>1 bench path on the one-GPU box: 2 ranks on cuda:0 over gloo (host-staged
# collectives), point-sharded configs[2] (weak: 2 x 32768 points) and sample-DP configs[4] (8 meshes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export GNOT_BENCH_BACKEND=gloo GNOT_BENCH_ONE_GPU=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 3 --warmup 2 --points 32768 > gpurun_out/be_shard.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 2 --steps 3 --warmup 2 --workload cfg5 --meshes 8 > gpurun_out/be_dp.log 2>&1
