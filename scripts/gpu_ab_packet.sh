#!/bin/bash
# packet walk + replay (option packet) — parity variants, then in-process A/B vs the traversal kernel
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
true > gpurun_out/packet_pytest.log

: > gpurun_out/ab_packet.log
echo start >> gpurun_out/ab_packet.log
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Glossy --spp 32 --depth 16 --reps 3 packet=0 packet=1 packet=2 packet=3 >> gpurun_out/ab_packet.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --synthetic 1000 --spp 16 --depth 8 --reps 3 packet=0 packet=1 packet=2 >> gpurun_out/ab_packet.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --synthetic 12500 --spp 16 --depth 8 --reps 2 packet=0 packet=1 packet=2 >> gpurun_out/ab_packet.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --spp 8 --depth 16 --reps 2 packet=0 packet=1 >> gpurun_out/ab_packet.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_packet.log
