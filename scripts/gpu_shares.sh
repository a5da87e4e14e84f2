#!/bin/bash
# One rank's share of an N-rank strong-scaling run, timed alone on one GPU (bench.py --share-of):
# BASELINE configs[1] (CornellBox 1024^2, 256 spp, depth 8) at N = 1, 2, 4, 8 and configs[4]'s
# 4096^2 image (4096 spp, depth 8) at N = 8 (512 frames per rank).  Lines -> gpurun_out/shares.jsonl
set -o pipefail
OUT=${OUT:-gpurun_out/shares.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" | tee -a "$OUT"; }
run --steps 5 --warmup 1 &&
for n in 2 4 8; do run --steps 5 --warmup 1 --share-of $n || exit 1; done &&
run --steps 3 --warmup 1 --width 4096 --height 4096 --spp 4096 --share-of 8 &&
run --steps 3 --warmup 1 --width 4096 --height 4096 --spp 4096 --share-of 8 --share-rank 7
