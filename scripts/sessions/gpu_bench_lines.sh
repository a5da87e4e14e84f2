#!/bin/bash
# Bench lines: the default (BASELINE configs[1]), without per-launch kernel events (their cost), and
# config 5's image (CornellBox 4096^2, depth 8) on one GPU at 64 spp -> gpurun_out/profiles/<TAG>_lines.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/profiles/${TAG}_lines.jsonl
mkdir -p gpurun_out/profiles
: > $OUT
run() {
  timeout -k 10 400 python3 bench.py "$@" > gpurun_out/line.log 2>&1
  rc=$?; echo "bench $* rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/line.log; exit $rc; }
  grep -h '^{' gpurun_out/line.log | tee -a $OUT | cut -c1-160
}
run --no-cpu-baseline
run --no-cpu-baseline --no-kernel-timing
run --no-cpu-baseline --width 4096 --height 4096 --spp 64 --steps 3
