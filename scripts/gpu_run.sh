#!/bin/bash
# GPU-box runner (one gpurun call = one invocation):  bash scripts/gpu_run.sh <tag> <step> [<step> ...]
# Steps run in order, each under its own time limit; the first failure ends the call (no GPU step runs
# after a fault, abort or timeout).  Outputs go to gpurun_out/<tag>_*.  '+' in a step argument = space.
#   tests[:<pytest -k expression>]   the -m gpu suite (or a subset)
#   file:<test file>[::<test>]       one test file / test
#   smoke                            __graft_entry__.smoke()
#   bench[:<bench.py args>]          one bench line -> <tag>_bench<n>.json
#   prof[:<bench.py args>]           rocprofv3 --kernel-trace --stats of a short bench run -> <tag>_prof<n>/
#   mb[:<microbench args>]           the kernel microbenchmark (lib/microbench)
#   mbx:<suffix>+<args>              an experimental build of it (lib/microbench_<suffix>)
#   dist:<nproc>+<bench args>        bench.py over <nproc> gloo ranks sharing cuda:0 (multi-GPU rehearsal)
set -o pipefail
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  arg=${arg//+/ }
  out=gpurun_out/${TAG}_${kind}${n}
  echo "[gpu_run] step $n: $kind $arg" >&2
  case $kind in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "$arg" > $out.log 2>&1
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $out.log 2>&1
      fi
      rc=$?; tail -4 $out.log ;;
    file)
      timeout -k 10 1000 python -u -m pytest "tests/$arg" -m gpu -x -v -s --timeout 900 --timeout-method thread > $out.log 2>&1
      rc=$?; tail -4 $out.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out.log 2>&1
      rc=$?; tail -2 $out.log ;;
    bench)
      timeout -k 10 600 python bench.py $arg > $out.json 2> $out.err
      rc=$?; tail -c 1500 $out.json; [ $rc -eq 0 ] || tail -20 $out.err ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$out" -o run \
        -- python3 bench.py --no-cpu-baseline $arg > $out.log 2>&1
      rc=$?; tail -3 $out.log ;;
    mb)
      timeout -k 10 300 gnot-replication_amd/lib/microbench $arg > $out.log 2>&1
      rc=$?; tail -30 $out.log ;;
    dist)  # dist:<nproc>+<bench args>: multi-process rehearsal on the one GPU (gloo, every rank on cuda:0)
      set -- $arg
      np=$1; shift
      GNOT_BENCH_BACKEND=gloo GNOT_BENCH_ONE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $np "$@" > $out.json 2> $out.err
      rc=$?; tail -c 1200 $out.json; [ $rc -eq 0 ] || tail -30 $out.err ;;
    mbx)   # an experimental microbench build: mbx:<suffix>+<args> runs lib/microbench_<suffix>
      set -- $arg
      sfx=$1; shift
      timeout -k 10 300 gnot-replication_amd/lib/microbench_$sfx "$@" > $out.log 2>&1
      rc=$?; tail -30 $out.log ;;
    *) echo "unknown step $kind" >&2; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "[gpu_run] step $n ($kind) failed rc=$rc" >&2
    exit $rc
  fi
done
echo "[gpu_run] done" >&2
