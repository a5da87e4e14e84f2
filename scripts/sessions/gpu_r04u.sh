#!/bin/bash
# Round 4: the full GPU suite with pooled leaf turns on the reference trees only (auto), then the config lines.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/profiles/r04u_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/r04u_pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_configs.sh r04u
