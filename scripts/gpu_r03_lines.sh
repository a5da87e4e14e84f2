#!/bin/bash
# round-3 config lines (BASELINE configs[2..3] at full spp) and the BVH-size sweep
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
bash scripts/gpu_configs.sh r03 || exit $?
SPP=16 bash scripts/gpu_sweep.sh r03 || exit $?
cp gpurun_out/r03_sweep.jsonl gpurun_out/profiles/r03_sweep.jsonl
