#!/bin/bash
# GPU box: parity tests, then bench + rocprofv3 summary.   bash scripts/gpu_test_bench.sh <tag> [bench args]
set -o pipefail
TAG=${1:-run}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_profile.sh "$TAG" "$@"
