set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "mailbox or tie or CornellBox-64" > gpurun_out/mb_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/mb_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/perf_variants.py --spp 64 --rounds 3 --variants ${AB_VARIANTS:-wf_nomb,wf_mb16} > gpurun_out/mb_ab.log 2>&1
rc=$?; cat gpurun_out/mb_ab.log; exit $rc
