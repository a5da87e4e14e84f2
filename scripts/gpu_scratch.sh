cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rP -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r02p_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02p_pytest.log; grep -E "ratio|FAILED" gpurun_out/r02p_pytest.log | head -40; exit $rc
