#!/bin/bash
# Full GPU test suite, then an in-process A/B of kernel variants (AB_VARIANTS, AB_SPP).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/check_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/check_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/perf_variants.py --spp ${AB_SPP:-64} --rounds 3 --variants ${AB_VARIANTS:-wf_nomb,wf_mb16} > gpurun_out/check_ab.log 2>&1
rc=$?; cat gpurun_out/check_ab.log; exit $rc
