#!/bin/bash
# Round 5: k_wf_trace_pre at 7 waves per SIMD (72 VGPRs, 32-84 B/lane of scratch) against 6, boat.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/tw7/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 > $P/r05ab_ab_tw7.log 2>&1
rc=$?; grep '"lib"' $P/r05ab_ab_tw7.log; [ $rc -eq 0 ] || exit $rc
