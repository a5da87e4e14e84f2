#!/bin/bash
# Round 6, final tree, part 2: PMC passes of configs[2] Mirror and Glossy and configs[3] MedievalBoat (their lines'
# executed-VALU figure, valu_exec), then the config lines and the BVH-size sweep.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 600 bash scripts/collect_traffic.sh --scene CornellBox-Mirror --spp 1024 --depth 16 > gpurun_out/r06k_traffic_mirror.log 2>&1 || exit $?
cp gpurun_out/profiles/traffic.json profiles/traffic.json
timeout -k 10 600 bash scripts/collect_traffic.sh --scene CornellBox-Glossy --spp 1024 --depth 16 > gpurun_out/r06k_traffic_glossy.log 2>&1 || exit $?
cp gpurun_out/profiles/traffic.json profiles/traffic.json
timeout -k 10 600 bash scripts/collect_traffic.sh --scene MedievalBoat --width 1920 --height 1080 --spp 512 --depth 16 > gpurun_out/r06k_traffic_boat.log 2>&1 || exit $?
cp gpurun_out/profiles/traffic.json profiles/traffic.json
bash scripts/gpu_configs.sh r06k || exit $?
SPP=16 bash scripts/gpu_sweep.sh r06k || exit $?
