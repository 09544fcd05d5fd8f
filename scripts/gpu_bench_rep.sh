#!/bin/bash
# Repeat the bench (no CPU baseline) to see run-to-run spread:  bash scripts/gpu_bench_rep.sh <n> [bench args...]
set -o pipefail
N=${1:-3}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/rep_$i.json 2> gpurun_out/rep_$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/rep_$i.json')); print('run $i', d['value'], d['ms_per_step'])"
done
