#!/bin/bash
# Round 6: the fused kernel's whole path chain in one launch (option persist, k_wf_persist): parity
# variants, in-process A/B, a rank's 1/8 share and the bench with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "persist or profile_records" --timeout 500 --timeout-method thread > gpurun_out/r06n_parity.log 2>&1 || exit $?
tail -1 gpurun_out/r06n_parity.log
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 400 python -u scripts/ab_libs.py $L $L@persist=1 $L $L@persist=1 --rounds 5 --async-torch --scene CornellBox --res 1024 --spp 64 --depth 8 > gpurun_out/r06n_ab_cornell.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/ab_libs.py $L $L@persist=1 --rounds 5 --async-torch --scene CornellBox-Mirror --res 1024 --spp 64 --depth 16 > gpurun_out/r06n_ab_mirror.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06n_ab_*.log
timeout -k 10 300 python -u bench.py --share-of 8 --no-cpu-baseline > gpurun_out/r06n_share8.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --share-of 8 --no-cpu-baseline --opt persist=1 > gpurun_out/r06n_share8_persist.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06n_n1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --opt persist=1 > gpurun_out/r06n_n1_persist.log 2>&1 || exit $?
for f in share8 share8_persist n1 n1_persist; do python3 -c "import json,sys; j=json.loads([l for l in open('gpurun_out/r06n_$f.log') if l.startswith('{')][-1]); print('$f', j['value'], j['ms_per_step'])"; done
