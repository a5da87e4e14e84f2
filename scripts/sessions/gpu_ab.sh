#!/bin/bash
# in-process env A/B only (no tests): scripts/gpu_ab.sh TAG [env_ab.py args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 500 python -u scripts/env_ab.py "$@" > gpurun_out/${TAG}_ab.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_ab.log; exit $rc
