#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench. Each GPU step has its own
# time limit; a crash/abort/timeout of any step ends the script (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  # any failure may be a GPU fault: start nothing more on the GPU in this call
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step build 600 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS:-}
if [ "${DIST_REHEARSAL:-0}" = "1" ]; then
  # 2 ranks sharing the one GPU, gloo: exercises bench.py's N>1 path (barrier, max-over-ranks)
  step bench_dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 \
      --backend gloo --windows 200000
fi
