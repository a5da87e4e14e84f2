#!/bin/bash
# Round 6: the leaf pass stress test with its output, the GPU suite on the one-alternative leaf
# remainders (default build), and in-process A/B of remainders off / one alternative / four.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_leafbvh.py -m gpu -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/r06b_leafbvh.log 2>&1 || exit $?
tail -20 gpurun_out/r06b_leafbvh.log
bash scripts/gpu_suite.sh r06b || exit $?
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py $L $L@leaf_skip=0 ablib/alt4/libpt_hip.so --rounds 5 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06b_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06b_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06b_ab_syn12k.log 2>&1 || exit $?
cat gpurun_out/r06b_ab_*.log
# the traversal kernel's turns (diagnostic build ablib/trace: make EXTRA=-DPT_TRACE_STATS=1)
timeout -k 10 300 python -u scripts/trace_stats.py ablib/trace/libpt_hip.so --scene CornellBox-Glossy --spp 8 > gpurun_out/r06b_trace_stats_glossy.json 2>&1 || exit $?
timeout -k 10 300 python -u scripts/trace_stats.py ablib/trace/libpt_hip.so --synthetic 12500 --spp 8 --depth 8 > gpurun_out/r06b_trace_stats_syn12k.json 2>&1 || exit $?
cat gpurun_out/r06b_trace_stats_*.json
