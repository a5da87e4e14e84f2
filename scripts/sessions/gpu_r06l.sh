#!/bin/bash
# Round 6: leaf turn followed by the node turn in the same turn (PT_LEAF_THEN_NODE=1 build) against
# HEAD (H) and the restructured default (L); the camera table on CornellBox.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
H=ablib/head/libpt_hip.so; T=ablib/ltn/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py $H $L $T $T@node_steps=2 $T@node_steps=8 --rounds 5 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06l_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06l_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06l_ab_syn12k.log 2>&1 || exit $?
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8 > gpurun_out/r06l_ab_syn100k.log 2>&1 || exit $?
ab --scene MedievalBoat --res 1024 --spp 16 --depth 16 > gpurun_out/r06l_ab_boat.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06l_ab_*.log
# the camera batches' table (k_wf_camtab) on the bench scene: HEAD against the tree
timeout -k 10 400 python -u scripts/ab_libs.py $H $L $H $L --rounds 5 --async-torch --scene CornellBox --res 1024 --spp 64 --depth 8 > gpurun_out/r06l_ab_cornell.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06l_ab_cornell.log
