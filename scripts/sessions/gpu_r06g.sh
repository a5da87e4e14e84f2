#!/bin/bash
# Round 6: several node steps per node turn (option node_steps): parity variants, in-process A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "nodesteps" --timeout 500 --timeout-method thread > gpurun_out/r06g_parity.log 2>&1 || exit $?
tail -1 gpurun_out/r06g_parity.log
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py ablib/base/libpt_hip.so $L $L@node_steps=2 $L@node_steps=3 --rounds 5 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06g_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06g_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06g_ab_syn12k.log 2>&1 || exit $?
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8 > gpurun_out/r06g_ab_syn100k.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06g_ab_*.log
timeout -k 10 400 python -u scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 8 --depth 16 --reps 3 'node_steps=1' 'node_steps=2' 'node_steps=3' > gpurun_out/r06g_ab_boat.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06g_ab_boat.log
