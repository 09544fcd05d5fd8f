#!/bin/bash
# r03x: fp32 chain-backward weight lead 3 (default) / 1 / 2 (GNOT_C2B_LEAD_X6 library builds), interleaved x2,
# the whole configs[2] fp32 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gnot-replication_amd/lib
for i in 1 2; do
  for v in "" _x1 _x2; do
    GNOT_LIB=$PWD/$L/libgnot_hip$v.so timeout -k 10 300 python bench.py --fp32-only --no-cpu-baseline \
      > gpurun_out/r03x_lead${v:-_x3}_$i.json 2> gpurun_out/r03x_lead${v:-_x3}_$i.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['class_ms_per_step'])" gpurun_out/r03x_lead${v:-_x3}_$i.json
  done
done
