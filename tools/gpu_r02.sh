#!/bin/bash
# Round-2 GPU session: build, gpu tests, then bench lines for the given configs.
# Every GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 4 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step build 600 make -s -j16 -C pymhealth_amd/csrc
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
for cfg in ${CONFIGS:-cfg2}; do
  step bench_$cfg 300 python bench.py --steps ${STEPS:-10} --warmup 2 --config $cfg --no-cpu-baseline
done
