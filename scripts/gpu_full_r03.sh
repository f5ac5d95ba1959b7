#!/bin/bash
# Full GPU suite + smoke + c2 bench + rocprof, then c1 c3 c4 c5 bench lines
# and kernel stats (round-3 refresh).  Stops at the first hard failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PROFILE=1 bash scripts/gpu_round.sh || exit $?
PROF=1 BSTEPS=20 bash scripts/gpu_all_cfg.sh
