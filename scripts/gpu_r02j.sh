#!/bin/bash
# chain2 counted-pipeline check: save-buffer dump vs the committed v2 kernels, GPU suite, determinism, microbench, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 180 python3 -u scripts/diag_dump_save.py 2048 gpurun_out/new.npz > gpurun_out/j_dump.log 2>&1 &&
GNOT_LIB=gnot-replication_amd/lib/libgnot_hip_v2.so timeout -k 10 180 python3 -u scripts/diag_dump_save.py 2048 gpurun_out/v2.npz >> gpurun_out/j_dump.log 2>&1 &&
python3 -c "
import numpy as np
a=np.load('gpurun_out/new.npz'); b=np.load('gpurun_out/v2.npz')
for k in a.files: print(k, np.abs(a[k]-b[k]).max(), (a[k]!=b[k]).sum())
" >> gpurun_out/j_dump.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/j_tests.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/diag_determinism.py 262144 > gpurun_out/j_det.log 2>&1 &&
timeout -k 10 120 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/j_mb.txt 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/j_bench.log 2>&1
