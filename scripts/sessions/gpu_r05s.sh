#!/bin/bash
# Round 5: Glossy's largest leaves (32-43 entries) resolved before the traversal? (big_leaf below
# 128 with the leaf pass forced or left to the probe), in process, same bits.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 scripts/env_ab.py --scene CornellBox-Glossy --width 1024 --height 1024 --spp 32 --depth 16 --reps 2 '' 'big_leaf=32' 'big_leaf=32,leaf_pre=1' 'big_leaf=24,leaf_pre=1' 'big_leaf=40,leaf_pre=1' 'big_leaf=32,leaf_pre=0' > $P/r05s_ab_glossy_pre.log 2>&1
rc=$?; grep variant $P/r05s_ab_glossy_pre.log; [ $rc -eq 0 ] || exit $rc
