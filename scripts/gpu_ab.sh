#!/bin/bash
# GPU box A/B of one tuning knob: parity tests once, then the bench (no CPU baseline) twice per value.
#   bash scripts/gpu_ab.sh <ENV_VAR> "<v1> <v2> ..." [bench args...]
set -o pipefail
VAR=$1; VALS=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_ab.log 2>&1
rc=$?
tail -3 gpurun_out/tests_ab.log
[ $rc -eq 0 ] || exit $rc
for v in $VALS; do
  for i in 1 2; do
    env "$VAR=$v" timeout -k 10 200 python -u bench.py --no-cpu-baseline --breakdown "$@" > gpurun_out/ab_${v}_$i.json 2> gpurun_out/ab_${v}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${v}_$i.json')); print('$VAR=$v run $i', d['value'], d['ms_per_step'])"
  done
done
