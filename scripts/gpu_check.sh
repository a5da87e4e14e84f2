#!/bin/bash
# GPU-box check: parity tests, smoke, short bench.  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
