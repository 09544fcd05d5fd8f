#!/bin/bash
# bf16 activation storage (bf16 mode soft-MoE chains + pgemm_b16_kernel): bf16 / walk / recompute tests,
# headline bf16 parity at 70k points, bench (fp32 + bf16 companion) and the bf16 A/B without bf16 storage
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_moe_walk.py tests/test_gpu_recompute.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1 &&
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_headline.py -m gpu -x -v -s -k bf16 --timeout 400 --timeout-method thread > gpurun_out/r03e_headline.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --breakdown > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err &&
GNOT_NO_B16S=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --dtype bf16 --fp32-only > gpurun_out/r03e_bench_nob16s.json 2> gpurun_out/r03e_bench_nob16s.err
