#!/bin/bash
# GPU box sweep of one environment setting over values, interleaved rounds: bench.py (no CPU baseline) per value.
#   bash scripts/gpu_env_sweep.sh <tag> <rounds> <VAR> "<v1> <v2> ..." [bench args...]
set -o pipefail
TAG=$1; R=$2; VAR=$3; VALS=$4; shift 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_${v}_$i.json 2> gpurun_out/${TAG}_${v}_$i.err || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_${v}_$i.json'))
b=d.get('bf16_mode',{})
print('$VAR=$v run $i', d['value'], d['ms_per_step'], 'bf16', b.get('ms_per_step'))"
  done
done
