#!/bin/bash
# A/B of library builds of the same sources (MHF_LIB): kernel ms per config, alternating
# builds REPS times.  LIBS="pymhealth_amd/libmhfeat.so pymhealth_amd/libmhfeat_nt.so"
# CONFIGS="cfg2 cfg3" FEATS_cfg2=mean (optional per-config feature override).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for i in $(seq ${REPS:-3}); do
  for c in ${CONFIGS:-cfg2 cfg3}; do
    for l in ${LIBS}; do
      fv="FEATS_$c"; extra=""
      [ -n "${!fv:-}" ] && extra="--features ${!fv}"
      MHF_LIB=$l timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 \
          --no-cpu-baseline $extra > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().split('\n')[-1]); print('$c', '$(basename $l)', '${!fv:-}', round(d['roofline']['kernel_ms'],4))"
    done
  done
done
