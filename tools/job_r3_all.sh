#!/bin/bash
# Round-3 GPU call: check job (diag, GPU suite, bench, old-code PPO profile), then the PPO job.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/job_r3_check.sh || exit $?
bash tools/job_r3_ppo.sh
