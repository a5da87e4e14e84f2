#!/bin/bash
# Round 6: the traversal's other knobs again with four node steps per node turn (pool runs, sort keys,
# sparse windows, the hit ring), in-process A/B on Glossy, synthetic 1k / 12.5k and the boat.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 500 python -u scripts/ab_libs.py $L $L@pool_run=2 $L@sort=64 $L@trace_sparse=0 $L@trace_ring=128 $L@node_steps=4,node_bias=3 $L --rounds 4 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06ac_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06ac_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06ac_ab_syn12k.log 2>&1 || exit $?
ab --scene MedievalBoat --res 1024 --spp 16 --depth 16 > gpurun_out/r06ac_ab_boat.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06ac_ab_*.log
