#!/bin/bash
# Full rocprofv3 set (trace + PMC passes) for every bench config; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r01b}
for c in ${CONFIGS:-cfg2 cfg3 cfg4 cfg5}; do
  bash tools/profile.sh ${TAG}_$c --config $c --steps 5 --warmup 1 || exit $?
done
