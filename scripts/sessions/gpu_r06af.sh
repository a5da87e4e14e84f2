#!/bin/bash
# Round 6, final: PMC of configs[2] Glossy (its traversal instance changed: pooled runs of 2), then
# the config lines and the BVH-size sweep.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 600 bash scripts/collect_traffic.sh --scene CornellBox-Glossy --spp 1024 --depth 16 > gpurun_out/r06af_traffic_glossy.log 2>&1 || exit $?
cp gpurun_out/profiles/traffic.json profiles/traffic.json
bash scripts/gpu_configs.sh r06af || exit $?
SPP=16 bash scripts/gpu_sweep.sh r06af || exit $?
