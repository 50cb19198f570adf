#!/bin/bash
# Round-end rehearsal on one GPU: smoke, default bench (with CPU baseline), a 2-rank gloo
# run of the bench's distributed path (both ranks on cuda:0), cfg3 / cfg5 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 2 "gpurun_out/$name.log" | cut -c1-600
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
step bench_default 400 python bench.py
step bench_gloo2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --no-cpu-baseline
for c in ${CONFIGS:-cfg3 cfg5}; do
  step bench_$c 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline
done
