#!/bin/bash
# Round 5, final tree: the whole GPU suite, smoke, the bench line (rocprof stats + trace union +
# PMC via gpu_round.sh), then the config lines and the sweep (scene-bytes figure now on each line).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh r05z || exit $?
bash scripts/gpu_configs.sh r05z || exit $?
