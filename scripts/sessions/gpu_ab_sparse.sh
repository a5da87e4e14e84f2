#!/bin/bash
# sparse trace windows for short queues (option trace_sparse=n): parity variants, then in-process A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -k "sparse" -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/sparse_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/sparse_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_sparse.log
V="trace_sparse=0 trace_sparse=1 trace_sparse=2 trace_sparse=4 trace_sparse=8"
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Glossy --spp 64 --depth 16 --reps 3 $V >> gpurun_out/ab_sparse.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 8 --depth 16 --reps 2 $V >> gpurun_out/ab_sparse.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --synthetic 12500 --spp 16 --depth 8 --reps 3 $V >> gpurun_out/ab_sparse.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --synthetic 1000000 --spp 4 --depth 8 --reps 2 $V >> gpurun_out/ab_sparse.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_sparse.log
