#!/bin/bash
# Round 5, final library: the BVH-size sweep (scene-bytes figure on each line) and the rank shares.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
bash scripts/gpu_sweep.sh r05ad || exit $?
cp gpurun_out/r05ad_sweep.jsonl gpurun_out/profiles/r05ad_sweep.jsonl
OUT=gpurun_out/profiles/r05ad_shares.jsonl bash scripts/gpu_shares.sh > gpurun_out/shares.log 2>&1
rc=$?; echo "shares rc=$rc"; exit $rc
