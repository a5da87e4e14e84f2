#!/bin/bash
# Round 6: pooled runs of 2 on every tree without big leaves (default): parity of the traversal
# variants and the fast trees, in-process A/B against runs of 4, the Glossy config line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fast_trees.py tests/test_gpu_config_bands.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r06ad_parity.log 2>&1 || exit $?
tail -1 gpurun_out/r06ad_parity.log
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py $L $L@pool_run=4 $L --rounds 4 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06ad_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06ad_ab_syn1k.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06ad_ab_*.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --scene CornellBox-Glossy --spp 1024 --depth 16 --steps 2 --warmup 1 > gpurun_out/r06ad_glossy.log 2>&1 || exit $?
grep '^{' gpurun_out/r06ad_glossy.log | tail -1 | cut -c1-200
