#!/bin/bash
# Round 4: k_wf_trace's 16-bit stacks in process (option stack16), then the config lines and the
# BVH-size sweep on the corrected SAH tree.  -> gpurun_out/profiles/r04b_*
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
AB=gpurun_out/profiles/r04b_ab_stack16.jsonl
: > $AB
ab() { timeout -k 10 300 python3 scripts/env_ab.py --reps 3 "$@" stack16=1 stack16=0 >> $AB 2>gpurun_out/ab.err; rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ab --scene CornellBox-Glossy --spp 32 --depth 16
ab --scene MedievalBoat --width 960 --height 540 --spp 8 --depth 16
ab --synthetic 1000 --spp 16 --depth 8
ab --synthetic 12500 --spp 16 --depth 8
ab --synthetic 100000 --spp 8 --depth 8
cat $AB
bash scripts/gpu_configs.sh r04b && cp gpurun_out/profiles/r04b_configs.jsonl gpurun_out/profiles/r04b_configs.jsonl.keep
SPP=16 bash scripts/gpu_sweep.sh r04b && cp gpurun_out/r04b_sweep.jsonl gpurun_out/profiles/r04b_sweep.jsonl
