#!/bin/bash
# Round 5: where the N = 8 rank share of configs[1] (32 frames, one 33.5 M-path batch) loses against
# N = 1: kernel trace of the share's steps (gaps, launch tails).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P gpurun_out/r05o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05o/kt -o run -- python3 bench.py --share-of 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05o/share.log 2>&1
rc=$?; grep '^{' gpurun_out/r05o/share.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --share-of 8 --steps 5 --warmup 1 --no-cpu-baseline > $P/r05o_share.log 2>&1
rc=$?; grep '^{' $P/r05o_share.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
