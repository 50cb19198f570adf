#!/bin/bash
# Repeated short benches of one config (run-to-run spread): REPS runs of CONFIG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in ${CONFIGS:-cfg3}; do
  for i in $(seq ${REPS:-3}); do
    timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rb.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/rb.log').read().strip().split('\n')[-1]); print('$c', round(d['roofline']['kernel_ms'],4))"
  done
done
