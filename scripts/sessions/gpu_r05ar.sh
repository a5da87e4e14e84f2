#!/bin/bash
# Round 5: the boat traversal knobs (leaf pass on) against AUTO, in process (same bits): node bias, pooled run
# length, sparse windows, coherence sort, trace ring.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 960 --spp 8 --depth 16 --reps 2 '' 'node_bias=1' 'node_bias=2' 'node_bias=8' 'pool_run=2' 'trace_sparse=0' 'trace_sparse=8' 'sort=64' 'sort=0' 'trace_ring=256' 'wf_trace_blocks=4096' > $P/r05ar_ab_glossy.log 2>&1
rc=$?; grep variant $P/r05ar_ab_glossy.log; exit $rc
