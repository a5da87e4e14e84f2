#!/bin/bash
# Round 5: the boat's traversal share — one more leaf resolved before it (big_leaf=100: the
# 125-entry leaf), pooled runs of 2, node bias 1 / 2 — in process, same bits.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 960 --spp 8 --depth 16 --reps 2 '' 'big_leaf=100' 'pool_run=2' 'node_bias=1' 'node_bias=2' 'leaf_blocks=2048' > $P/r05v_ab_boat_trace.log 2>&1
rc=$?; grep variant $P/r05v_ab_boat_trace.log; [ $rc -eq 0 ] || exit $rc
