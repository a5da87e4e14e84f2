#!/bin/bash
# Round 5, final library (merged pass chunks, refine terms by bpermute): whole GPU suite, smoke, bench (+ rocprof stats,
# trace union, PMC via gpu_round.sh), config lines.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh r05am || exit $?
bash scripts/gpu_configs.sh r05am || exit $?
