#!/bin/bash
# GPU suite, then bench lines for $CONFIGS (kernel ms); stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-cfg2}; do
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { tail -5 gpurun_out/bench_$c.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$c.log').read().strip().split('\n')[-1]); r=d['roofline']; print('$c', d['config']['kernel'], round(r['kernel_ms'],4), 'ms', round(r['achieved']), 'GB/s', round(r['frac'],3))"
done
