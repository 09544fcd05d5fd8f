#!/bin/bash
# GPU box iteration: kernel microbenchmark, parity tests, bench line (no profile).
#   bash scripts/gpu_iter.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-it}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./gnot-replication_amd/lib/microbench > gpurun_out/mb_$TAG.txt 2>&1 || exit 1
cat gpurun_out/mb_$TAG.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --breakdown --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json; grep breakdown gpurun_out/bench_$TAG.err
