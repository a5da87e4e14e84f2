#!/bin/bash
# Round 4: with the shared chunk walk, do leaf chunks pay on mid-size leaves too?  Glossy (leaves of
# 40-61 entries), the 100k and 1M synthetic scenes (leaves of 30-127): scenes created with leaf
# chunks from 32 / 64 entries (option leaf_bvh; the big-leaf threshold follows it) against the
# default (128).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
OUT=gpurun_out/profiles/r04l_ab_leafbvh.jsonl
: > $OUT
for args in "--scene CornellBox-Glossy --spp 16 --depth 16" "--synthetic 100000 --spp 4 --depth 8" "--synthetic 1000000 --spp 2 --depth 8"; do
  for lb in 128 64 32 16; do
    echo "{\"args\": \"$args\", \"leaf_bvh\": $lb}" >> $OUT
    timeout -k 10 300 python3 scripts/env_ab.py $args --reps 3 --scene-opt leaf_bvh=$lb big_leaf=$lb >> $OUT 2>gpurun_out/ab.err
    rc=$?; echo "leaf_bvh=$lb $args rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
cat $OUT
