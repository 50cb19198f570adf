#!/bin/bash
# End-of-round GPU session, part 1: build, the whole gpu test suite, smoke(), the default
# bench line (with cpu_baseline) and the other BASELINE configs. Any failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step build 600 make -s -j16 -C pymhealth_amd/csrc
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_default 400 python bench.py
for cfg in ${CONFIGS:-cfg3 cfg4 cfg5}; do
  step bench_$cfg 400 python bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline
done
echo done
