#!/bin/bash
# GPU-box: parity tests then kernel A/B.  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python scripts/perf_variants.py --spp 64 --variants auto,wavefront_lean4_fastrcp,wavefront_lean16_fastrcp "$@" > gpurun_out/perf.log 2>&1
rc=$?; echo "perf rc=$rc"; cat gpurun_out/perf.log | grep -v amdgpu.ids
exit $rc
