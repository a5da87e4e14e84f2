#!/bin/bash
# Round 4: the RCCL branch of pt_render_multi on the one-GPU box (a one-rank communicator, option
# reduce=rccl) and the bench's native multi-GPU mode through it; then the GPU tests the round's
# last product changes touch.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k "multi or leaf or boat or big or fast_trees or config_bands" > gpurun_out/profiles/r04r_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/r04r_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --native-multi --gpus 1 --reduce rccl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/profiles/r04r_bench_native_rccl1.log 2>&1
rc=$?; echo "native rccl bench rc=$rc"; grep "^{" gpurun_out/profiles/r04r_bench_native_rccl1.log | cut -c1-300
