#!/bin/bash
# Round 6: node_steps default 3; parity of the node-step variants, in-process A/B of 1/3/4/6/8
# (traversal scenes, the boat, SAH trees, a small megakernel render).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "nodesteps or wavefront_default or mega_default or Glossy" --timeout 500 --timeout-method thread > gpurun_out/r06h_parity.log 2>&1 || exit $?
tail -1 gpurun_out/r06h_parity.log
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py ablib/base/libpt_hip.so $L@node_steps=1 $L $L@node_steps=4 $L@node_steps=6 $L@node_steps=8 --rounds 5 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06h_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06h_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8 > gpurun_out/r06h_ab_syn100k.log 2>&1 || exit $?
ab --scene CornellBox-Glossy --res 256 --spp 4 --depth 16 > gpurun_out/r06h_ab_glossy_small_mega.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06h_ab_*.log
V="node_steps=1 node_steps=3 node_steps=4 node_steps=6 node_steps=8"
timeout -k 10 400 python -u scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 8 --depth 16 --reps 3 $V > gpurun_out/r06h_ab_boat.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/env_ab.py --scene CornellBox-Glossy --bvh sah --spp 32 --depth 16 --reps 3 $V > gpurun_out/r06h_ab_glossy_sah.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/env_ab.py --scene MedievalBoat --bvh sah --width 1920 --height 1080 --spp 32 --depth 16 --reps 3 $V > gpurun_out/r06h_ab_boat_sah.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06h_ab_boat*.log gpurun_out/r06h_ab_glossy_sah.log
