#!/bin/bash
# Round 5, verdict r04 item 5: AUTO's per-scene choices against each alternative on scenes outside
# the tuning set (CornellBox-Sphere, CornellBox2 with every mesh), in process, same bits; plus the
# new band tests for both.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_config_bands.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "sphere or cornellbox2" > $P/r05d_pytest_bands.log 2>&1
rc=$?; tail -3 $P/r05d_pytest_bands.log; [ $rc -eq 0 ] || exit $rc
OUT=$P/r05d_auto_ab.log
: > $OUT
timeout -k 10 600 python3 scripts/env_ab.py --scene CornellBox-Sphere --width 1024 --height 1024 --spp 32 --depth 16 --reps 3 \
  '' 'pool_run=2' 'pool_run=4' 'node_bias=1' 'node_bias=4' 'leaf_pool=0' 'big_leaf=32' 'kernel=mega' 'sort=0' >> $OUT 2>&1
rc=$?; echo "sphere rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/env_ab.py --scene CornellBox2 --all-meshes --width 1024 --height 1024 --spp 8 --depth 16 --reps 3 \
  '' 'pool_run=2' 'pool_run=4' 'node_bias=1' 'node_bias=4' 'big_leaf=64' 'big_leaf=512' 'leaf_pre=0' 'kernel=mega' >> $OUT 2>&1
rc=$?; echo "cb2 rc=$rc"; grep -o '"variant": "[^"]*", "scene": "[^"]*", "ms": [0-9.]*, "msamples_s": [0-9.]*' $OUT; [ $rc -eq 0 ] || exit $rc
# verdict r04 item 4: the N = 8 rank share of configs[1] (32 frames of CornellBox 1024^2, depth 8) —
# one batch, so its launch tails weigh more per sample; parts on more streams to fill them
OUT2=$P/r05d_share_ab.log
timeout -k 10 600 python3 scripts/env_ab.py --scene CornellBox --width 1024 --height 1024 --spp 32 --depth 8 --reps 5 \
  '' 'parts=3' 'parts=4' > $OUT2 2>&1
rc=$?; echo "share rc=$rc"; grep -o '"variant": "[^"]*", "scene": "[^"]*", "ms": [0-9.]*, "msamples_s": [0-9.]*' $OUT2; exit $rc
