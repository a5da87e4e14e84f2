#!/bin/bash
# Parity suite + smoke + one bench line (+ optional extra command): the quick GPU check after a change.
# usage: gpu_check.sh TAG [extra script]   -> gpurun_out/profiles/TAG_pytest_gpu.log, TAG_bench.json
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-check}
mkdir -p gpurun_out/profiles
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/profiles/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/${TAG}_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/profiles/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/profiles/${TAG}_bench.log > gpurun_out/profiles/${TAG}_bench.json; cut -c1-200 gpurun_out/profiles/${TAG}_bench.json
if [ $rc -ne 0 ]; then exit $rc; fi
if [ $# -ge 2 ]; then bash "$2"; fi
