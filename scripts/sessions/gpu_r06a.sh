#!/bin/bash
# Round 6, leaf remainders (option leaf_skip): the GPU suite, then in-process A/B on/off on Glossy
# (configs[2]), the synthetic sweep's trees and the boat.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_suite.sh r06a || exit $?
ab() { timeout -k 10 300 python -u scripts/env_ab.py "$@"; }
ab --scene CornellBox-Glossy --spp 32 --depth 16 --reps 3 'leaf_skip=1' 'leaf_skip=0' > gpurun_out/r06a_ab_glossy.log 2>&1 || exit $?
ab --synthetic 1000 --spp 16 --depth 8 --reps 3 'leaf_skip=1' 'leaf_skip=0' > gpurun_out/r06a_ab_syn1k.log 2>&1 || exit $?
ab --synthetic 12500 --spp 16 --depth 8 --reps 3 'leaf_skip=1' 'leaf_skip=0' > gpurun_out/r06a_ab_syn12k.log 2>&1 || exit $?
ab --synthetic 100000 --spp 8 --depth 8 --reps 3 'leaf_skip=1' 'leaf_skip=0' > gpurun_out/r06a_ab_syn100k.log 2>&1 || exit $?
ab --scene MedievalBoat --width 1920 --height 1080 --spp 8 --depth 16 --reps 2 'leaf_skip=1' 'leaf_skip=0' > gpurun_out/r06a_ab_boat.log 2>&1 || exit $?
cat gpurun_out/r06a_ab_*.log
# the fused kernel's phases (diagnostic build of the same sources, ablib/phase: make EXTRA=-DPT_PHASE_STATS=1)
timeout -k 10 300 python -u scripts/phase_stats.py ablib/phase/libpt_hip.so > gpurun_out/r06a_phase_stats.json 2> gpurun_out/r06a_phase_stats.err || exit $?
cat gpurun_out/r06a_phase_stats.json
# the bench line (now with the GPU's clock / power state)
timeout -k 10 300 python -u bench.py > gpurun_out/r06a_bench.log 2>&1 || exit $?
tail -c 3000 gpurun_out/r06a_bench.log
