#!/bin/bash
# Diagnostic: memory floor of the tile kernel (pass 1 only: mean) on the cfg2 / cfg3 data.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in cfg2 cfg3; do
  timeout -k 10 120 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --features mean > gpurun_out/b.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().split('\n')[-1]); r=d['roofline']; print('$c mean-only', round(r['kernel_ms'],4), 'ms', round(r['achieved'],1), 'GB/s')"
done
