#!/bin/bash
# Round-3 session e: new division-fallback parity test, the whole GPU suite, smoke, the
# default bench (with the CPU baseline), the self-launched 2-rank bench, every workload's
# bench line, and rocprofv3 passes of cfg2 / cfg3 / cfgidx on this build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 2 "gpurun_out/$name.log" | cut -c1-400
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step tests_div 600 $PYT -m gpu tests/test_gpu_parity.py -k "division"
step tests_gpu 1000 $PYT -m gpu tests
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
step bench_default 400 python bench.py
step bench_gpus2 300 python bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --no-cpu-baseline
for c in ${CONFIGS:-cfg3 cfg4 cfg5 cfg2f64 cfgidx}; do
  step bench_$c 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline
done
if [ "${PROF:-1}" = "1" ]; then
  bash tools/profile.sh r03e_cfg2 --config cfg2 --steps 5 --warmup 1 > gpurun_out/prof_cfg2.log 2>&1 || exit 1
  bash tools/profile.sh r03e_cfg3 --config cfg3 --steps 5 --warmup 1 > gpurun_out/prof_cfg3.log 2>&1 || exit 1
fi
