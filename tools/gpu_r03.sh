#!/bin/bash
# Round-3 GPU session: the new / changed GPU tests first, then the whole GPU suite, smoke,
# the default bench line and the self-launched 2-rank bench (gloo, both ranks on cuda:0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/$name.log" | cut -c1-800
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
if [ -n "${TESTS:-}" ]; then step tests_new 900 $PYT -m gpu $TESTS; fi
if [ "${FULL:-1}" = "1" ]; then step tests_gpu 1000 $PYT -m gpu tests; fi
if [ "${SMOKE:-1}" = "1" ]; then step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"; fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench_default 400 python bench.py
  step bench_gpus2 300 python bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --no-cpu-baseline
fi
for c in ${CONFIGS:-}; do
  step bench_$c 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline
done
