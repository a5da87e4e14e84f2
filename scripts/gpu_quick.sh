cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02a_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r02a_bench.log 2>&1; rc=$?; grep '^{' gpurun_out/r02a_bench.log | cut -c1-400; exit $rc
