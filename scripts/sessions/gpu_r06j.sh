#!/bin/bash
# Round 6: node-step rule A/B (PT_NODE_STEP_RULE=1 build: a node turn's further steps end where the
# loop's next turn would be a leaf turn) against the default, at node_steps 4 and 8.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
R=ablib/rule1/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py $L $R $L@node_steps=8 $R@node_steps=8 --rounds 5 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06j_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06j_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06j_ab_syn12k.log 2>&1 || exit $?
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8 > gpurun_out/r06j_ab_syn100k.log 2>&1 || exit $?
ab --scene MedievalBoat --res 1024 --spp 16 --depth 16 > gpurun_out/r06j_ab_boat.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06j_ab_*.log
