#!/bin/bash
# Round 6: streaming regeneration in the fused kernel (option regen = camera batches per region per
# extension launch): parity variants, in-process A/B, a rank's 1/8 share and N = 1.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "regen" --timeout 500 --timeout-method thread > gpurun_out/r06r_parity.log 2>&1 || exit $?
tail -1 gpurun_out/r06r_parity.log
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 400 python -u scripts/ab_libs.py $L $L@regen=64 $L@regen=128 $L@regen=256 $L@regen=128,parts=1 $L --rounds 3 --async-torch --scene CornellBox --res 1024 --spp 32 --depth 8 > gpurun_out/r06r_ab_share.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/ab_libs.py $L $L@regen=128 $L@regen=256 $L@regen=512 $L --rounds 3 --async-torch --scene CornellBox --res 1024 --spp 256 --depth 8 > gpurun_out/r06r_ab_n1.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06r_ab_*.log
