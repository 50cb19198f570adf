#!/bin/bash
# Kernel time of one config for nested feature sets (what each pass / chain costs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
C=${CONFIG:-cfg2}
for f in ${SETS:-mean mean,zero_crossings mean,var32 mean,var mean,var,skewness,kurtosis,zero_crossings}; do
  timeout -k 10 120 python bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --features $f > gpurun_out/fd.log 2>&1 || { tail -3 gpurun_out/fd.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/fd.log').read().strip().split('\n')[-1]); print('$C', '$f', round(d['roofline']['kernel_ms'],4))"
done
