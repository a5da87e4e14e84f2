#!/bin/bash
# Round 6: kernel trace of the traversal pipeline (Glossy 1024^2, 64 spp, depth 16): how long the
# shade kernels take against the traversal, per launch and per depth.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06e_glossy_kt -o run -- python3 bench.py --scene CornellBox-Glossy --spp 64 --depth 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r06e_glossy_kt.log 2>&1 || exit $?
ls gpurun_out/r06e_glossy_kt
