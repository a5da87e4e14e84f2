#!/bin/bash
# Round 5, the tree as it will be left: the whole GPU suite, smoke and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 600 --timeout-method thread > $P/r05as_pytest_gpu.log 2>&1
rc=$?; tail -2 $P/r05as_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 __graft_entry__.py smoke > $P/r05as_smoke.log 2>&1
rc=$?; tail -1 $P/r05as_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $P/r05as_bench.json 2> $P/r05as_bench.err
rc=$?; cut -c1-200 $P/r05as_bench.json; exit $rc
