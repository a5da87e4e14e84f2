#!/bin/bash
# Round 6: why k_wf_trace's lanes idle (ring-blocked vs tail); the late flush (option trace_late)
# checked against the oracle and A/B'd in process against the committed library (ablib/base); where a
# rank's 1/8 share loses against N = 1 (kernel trace of the share).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/trace_stats.py ablib/trace/libpt_hip.so --scene CornellBox-Glossy --spp 8 > gpurun_out/r06c_trace_stats_glossy.json 2>&1 || exit $?
timeout -k 10 300 python -u scripts/trace_stats.py ablib/trace/libpt_hip.so --synthetic 1000 --spp 8 --depth 8 > gpurun_out/r06c_trace_stats_syn1k.json 2>&1 || exit $?
grep -A3 '"blocked"\|"starved"' gpurun_out/r06c_trace_stats_glossy.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "late or skip" --timeout 500 --timeout-method thread > gpurun_out/r06c_parity_late.log 2>&1 || exit $?
tail -2 gpurun_out/r06c_parity_late.log
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
ab() { timeout -k 10 400 python -u scripts/ab_libs.py ablib/base/libpt_hip.so $L $L@trace_late=1 --rounds 5 --async-torch "$@"; }
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16 > gpurun_out/r06c_ab_glossy.log 2>&1 || exit $?
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8 > gpurun_out/r06c_ab_syn1k.log 2>&1 || exit $?
ab --scene synthetic-12500 --res 1024 --spp 16 --depth 8 > gpurun_out/r06c_ab_syn12k.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06c_ab_*.log
B="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r06c_n1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $B --share-of 8 > gpurun_out/r06c_share8.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/r06c_n1.log gpurun_out/r06c_share8.log | head -4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06c_share_kt -o run -- python3 bench.py $B --share-of 8 > gpurun_out/r06c_share8_kt.log 2>&1 || exit $?
ls -R gpurun_out/r06c_share_kt | head
