#!/bin/bash
# A/B of (library, environment) variants on one config: kernel ms, REPS rounds.
# VARIANTS="libA.so:ENV=1 libB.so:" CONFIG=cfg5 REPS=2 tools/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
  for v in ${VARIANTS}; do
    lib=${v%%:*}; envs=${v#*:}
    env MHF_LIB=$lib ${envs:+${envs//,/ }} timeout -k 10 120 python bench.py --config ${CONFIG:-cfg5} --steps 20 --warmup 3 \
        --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().split('\n')[-1]); print('${CONFIG:-cfg5}', '$v', round(d['roofline']['kernel_ms'],4))"
  done
done
