#!/bin/bash
# r03z: bf16-storage backward pair mode + final-tree validation: microbench, the whole GPU suite, smoke, the default bench line, rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/r03z_mb.log 2>&1 || { cat gpurun_out/r03z_mb.log; exit 1; }
grep chain gpurun_out/r03z_mb.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r03z_tests.log 2>&1 || { tail -40 gpurun_out/r03z_tests.log; exit 1; }
tail -2 gpurun_out/r03z_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03z_smoke.log 2>&1 || { tail -20 gpurun_out/r03z_smoke.log; exit 1; }
tail -1 gpurun_out/r03z_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r03z_bench.json 2> gpurun_out/r03z_bench.err || { tail -20 gpurun_out/r03z_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03z_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac_pipe'], d['roofline']['traffic'], d['bf16_mode']['value'], d['bf16_mode']['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_r03z" -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_r03z.log 2>&1 || { tail -20 gpurun_out/prof_r03z.log; exit 1; }
echo done
