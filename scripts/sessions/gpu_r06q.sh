#!/bin/bash
# Round 6: the lean traversal's turn policy again with four node steps per node turn: node_bias 2 / 4
# (default) / 8 / 16, in-process A/B on the traversal scenes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py $L $L@node_bias=2 $L@node_bias=8 $L@node_bias=16 $L --rounds 5 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06q_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06q_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06q_ab_syn12k.log 2>&1 || exit $?
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8 > gpurun_out/r06q_ab_syn100k.log 2>&1 || exit $?
ab --scene MedievalBoat --res 1024 --spp 16 --depth 16 > gpurun_out/r06q_ab_boat.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06q_ab_*.log
