#!/bin/bash
# Round 5, final library (the pass's lean check): whole GPU suite, smoke, bench (+ rocprof stats,
# trace union, PMC via gpu_round.sh), config lines.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh r05ac || exit $?
bash scripts/gpu_configs.sh r05ac || exit $?
