#!/bin/bash
# bf16 mode: dZ stored as RNE bf16 by the chain backward (the wide weight-gradient kernel's one-piece
# operand bits); GPU suite (bf16 parity at 1e-2 included), configs[2] bench with the bf16 companion
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bd_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --breakdown > gpurun_out/bd_bench.json 2> gpurun_out/bd_bench.err
