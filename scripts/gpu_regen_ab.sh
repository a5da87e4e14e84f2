cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_parity.py -k "bench_config or config1 or multi_batch or render_accum or auto_ or large or gen or persist" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r02d_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02d_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/env_ab.py "$@" 2>&1 | tee gpurun_out/r02d_ab.log
