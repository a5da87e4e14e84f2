#!/bin/bash
# per-launch kernel durations of a traversal-scene render (which bounce costs what)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
SCENE=${1:-CornellBox-Glossy}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lp_$SCENE -o run -- python3 bench.py --scene $SCENE --spp 16 --depth 16 --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing > gpurun_out/lp_$SCENE.log 2>&1 || exit $?
python3 scripts/launch_profile.py gpurun_out/lp_$SCENE/run_kernel_trace.csv
