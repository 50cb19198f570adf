#!/bin/bash
# rocprofv3 passes on the bench workload (run on the GPU box):
#   1. kernel trace + stats (durations)
#   2..n. PMC passes, each in its own run (kernel trace only alongside, as required)
# Usage: tools/profile.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
KRE=${KRE:-tile_kernel|tile64_kernel|tile64_stream_kernel|moments_generic|span_kernel|spectral_kernel|spectral_wave_kernel|spectral_reg_kernel}
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" rocprofv3 "$@" --kernel-include-regex "$KRE" --output-format csv \
      -d "$OUT/$name" -o "$name" -- python3 bench.py --no-cpu-baseline "${BENCH[@]}" \
      > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$OUT/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
BENCH=("$@")
run trace 300 --kernel-trace --stats
[ "${QUICK:-0}" = "1" ] && { run sq 300 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE; run sq2 300 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES; run icache 300 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQC_TC_INST_REQ SQC_ICACHE_MISSES_DUPLICATE; exit 0; }
run fetch 300 --kernel-trace --pmc FETCH_SIZE
run write 300 --kernel-trace --pmc WRITE_SIZE
run sq 300 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run sq2 300 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES
run icache 300 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQC_TC_INST_REQ SQC_ICACHE_MISSES_DUPLICATE
