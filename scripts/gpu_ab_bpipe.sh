#!/bin/bash
# batch pipelining (option batch_pipe): parity, then in-process A/B on the benchmarked scenes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bench_config.py -q -k "batch_pipe or multi_batch" -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/bpipe_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/bpipe_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_bpipe.log
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox --spp 256 --depth 8 --reps 3 batch_pipe=0 batch_pipe=1 >> gpurun_out/ab_bpipe.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Glossy --spp 64 --depth 16 --reps 3 batch_pipe=0 batch_pipe=1 >> gpurun_out/ab_bpipe.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Mirror --spp 64 --depth 8 --reps 3 batch_pipe=0 batch_pipe=1 >> gpurun_out/ab_bpipe.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 16 --depth 16 --reps 2 batch_pipe=0 batch_pipe=1 >> gpurun_out/ab_bpipe.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --synthetic 100000 --spp 64 --depth 8 --reps 3 batch_pipe=0 batch_pipe=1 >> gpurun_out/ab_bpipe.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_bpipe.log
