#!/bin/bash
# Round-end style GPU session: parity tests, smoke, bench, rocprofv3 kernel trace of the bench,
# PMC traffic + VALU issue, bench again (reads them).  Summaries -> gpurun_out/profiles/<tag>_*
# (copy into profiles/).  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out/profiles
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rP -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/profiles/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/profiles/${TAG}_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bench_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_kt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
cp gpurun_out/bench_kt/run_kernel_stats.csv gpurun_out/profiles/${TAG}_bench_kernel_stats.csv
grep "^{" gpurun_out/bench_kt.log > gpurun_out/profiles/${TAG}_bench_under_rocprof.json || true
# the kernel's busy time from the trace itself (union of its dispatch intervals), for bench.py
cp profiles/trace_union.json gpurun_out/profiles/trace_union.json 2>/dev/null || true
python3 scripts/trace_union.py gpurun_out/bench_kt/run_kernel_trace.csv gpurun_out/profiles/${TAG}_bench_under_rocprof.json \
  gpurun_out/profiles/trace_union.json > gpurun_out/profiles/${TAG}_trace_union.log 2>&1
rc=$?; echo "trace union rc=$rc"; grep busy_ms gpurun_out/profiles/${TAG}_trace_union.log
cp gpurun_out/profiles/trace_union.json profiles/trace_union.json 2>/dev/null || true
# VALU issue calibration (the traffic summary below applies it)
timeout -k 10 400 bash scripts/calibrate_valu.sh > gpurun_out/profiles/${TAG}_valu_calibration.log 2>&1
rc=$?; echo "valu calibration rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
cp gpurun_out/profiles/valu_calibration.json profiles/valu_calibration.json
timeout -k 10 900 bash scripts/collect_traffic.sh
rc=$?; echo "traffic rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
# this box's copy of the tree: let the second bench read the traffic just measured
cp gpurun_out/profiles/traffic.json profiles/traffic.json
timeout -k 10 300 python bench.py > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench2 rc=$rc"; grep "^{" gpurun_out/bench2.log | cut -c1-300
grep "^{" gpurun_out/bench2.log > gpurun_out/profiles/${TAG}_bench.json || true
cp gpurun_out/bench.log gpurun_out/profiles/${TAG}_bench.log
exit $rc
