#!/bin/bash
# Round 6: k_wf_persist, grid from its own occupancy, and capped grids (is the persistent grid
# resident?): in-process A/B on CornellBox.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 500 python -u scripts/ab_libs.py $L $L@persist=1 $L@persist=1,wf_trace_blocks=1792 $L@persist=1,wf_trace_blocks=1536 $L@persist=1,wf_trace_blocks=1024 $L@persist=1,wf_trace_blocks=512 $L@wf_trace_blocks=1024 --rounds 3 --async-torch --scene CornellBox --res 1024 --spp 64 --depth 8 > gpurun_out/r06p_ab_cornell.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06p_ab_cornell.log
