#!/bin/bash
# Round 6: with pooled runs of 2 by default on trees without big leaves, the turn policy again:
# node bias 1 (run-2 default) / 2 / 4 and node steps 3 / 6, in-process A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 500 python -u scripts/ab_libs.py $L $L@node_bias=2 $L@node_bias=4 $L@node_steps=3 $L@node_steps=6 $L --rounds 4 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06ae_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06ae_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06ae_ab_syn12k.log 2>&1 || exit $?
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8 > gpurun_out/r06ae_ab_syn100k.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06ae_ab_*.log
