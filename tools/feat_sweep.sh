#!/bin/bash
# Diagnostic: cfg2 kernel time for growing feature subsets (memory floor vs compute).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for f in mean mean,zero_crossings mean,var32 mean,var,skewness,kurtosis,zero_crossings; do
  timeout -k 10 120 python bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --features $f > gpurun_out/b.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().split('\n')[-1]); print('$f', round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],3))"
done
