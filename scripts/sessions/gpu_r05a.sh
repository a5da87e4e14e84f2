#!/bin/bash
# Round 5, first session: the round-4 tree plus the RCCL group fix, the advisor's device fixes
# (wave LDS fences, keys only for lean flavours, node bias per instance, +inf hits in pooled turns),
# the SAH emitter leaf and its GPU test, the bench's host copy and valu_alg: GPU suite, smoke,
# bench, the boat's config line (baseline before the big-leaf pre-pass).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 600 --timeout-method thread > $P/r05a_pytest_gpu.log 2>&1
rc=$?; tail -3 $P/r05a_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 __graft_entry__.py smoke > $P/r05a_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $P/r05a_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $P/r05a_bench.json 2> $P/r05a_bench.err
rc=$?; echo "bench rc=$rc"; cat $P/r05a_bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene MedievalBoat --width 1920 --height 1080 --spp 512 --depth 16 > $P/r05a_boat.json 2>&1
rc=$?; echo "boat rc=$rc"; cut -c1-300 $P/r05a_boat.json; exit $rc
