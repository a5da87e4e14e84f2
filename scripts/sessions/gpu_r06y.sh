#!/bin/bash
# Round 6, final tree, part 1: the round-end set (GPU suite, smoke, bench, rocprofv3 kernel trace +
# trace union, VALU calibration, PMC traffic, bench again with the fresh PMC).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh r06y || exit $?
