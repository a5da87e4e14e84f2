set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 600 python -u -m pytest tests/test_gpu_config_bands.py tests/test_gpu_dist.py tests/test_gpu_multi.py -v -s -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/r03b_bands.log 2>&1
rc=$?; echo "bands rc=$rc"; grep -E "PASSED|FAILED|product tree|passed|failed" gpurun_out/r03b_bands.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 bash scripts/calibrate_valu.sh > gpurun_out/r03b_valucal.log 2>&1
rc=$?; echo "valucal rc=$rc"; tail -30 gpurun_out/r03b_valucal.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bench_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_kt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep "^{" gpurun_out/bench_kt.log > gpurun_out/profiles/r03b_bench_under_rocprof.json
python3 scripts/trace_union.py gpurun_out/bench_kt/run_kernel_trace.csv gpurun_out/profiles/r03b_bench_under_rocprof.json gpurun_out/profiles/trace_union.json
