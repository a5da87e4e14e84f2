#!/bin/bash
# Round 6: why k_wf_trace's lanes idle (ring-blocked vs tail), and where a rank's 1/8 share loses
# against N = 1 (kernel trace of the share).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/trace_stats.py ablib/trace/libpt_hip.so --scene CornellBox-Glossy --spp 8 > gpurun_out/r06c_trace_stats_glossy.json 2>&1 || exit $?
timeout -k 10 300 python -u scripts/trace_stats.py ablib/trace/libpt_hip.so --synthetic 1000 --spp 8 --depth 8 > gpurun_out/r06c_trace_stats_syn1k.json 2>&1 || exit $?
cat gpurun_out/r06c_trace_stats_*.json | grep -A3 '"blocked"\|"starved"\|"loop"'
B="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r06c_n1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $B --share-of 8 > gpurun_out/r06c_share8.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/r06c_n1.log gpurun_out/r06c_share8.log | head -4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06c_share_kt -o run -- python3 bench.py $B --share-of 8 > gpurun_out/r06c_share8_kt.log 2>&1 || exit $?
ls gpurun_out/r06c_share_kt
