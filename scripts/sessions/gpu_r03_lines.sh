#!/bin/bash
# round-3 config lines (BASELINE configs[2..3] at full spp) and the BVH-size sweep
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out/profiles
bash scripts/gpu_configs.sh $TAG || exit $?
SPP=16 bash scripts/gpu_sweep.sh $TAG || exit $?
cp gpurun_out/${TAG}_sweep.jsonl gpurun_out/profiles/${TAG}_sweep.jsonl
