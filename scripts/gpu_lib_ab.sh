#!/bin/bash
# GPU box A/B of two builds of libgnot_hip.so (GNOT_LIB), interleaved: bench.py (no CPU baseline) per build,
# `rounds` times.   bash scripts/gpu_lib_ab.sh <tag> <rounds> <lib A> <lib B> [bench args...]
set -o pipefail
TAG=$1; R=$2; A=$3; B=$4; shift 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for lib in "$A" "$B"; do
    n=$(basename "$lib" .so)
    GNOT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_${n}_$i.json 2> gpurun_out/${TAG}_${n}_$i.err || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_${n}_$i.json'))
b=d.get('bf16_mode',{})
print('$n run $i', d['value'], d['ms_per_step'], d['roofline']['class_ms_per_step'], 'bf16', b.get('ms_per_step'))"
  done
done
