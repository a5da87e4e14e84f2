#!/bin/bash
# Round 6: the step's readback by pt_readback_async (16 blocks) against torch's copy_ (the runtime's
# ~512-block blit kernel beside the next render): readback tests, then the bench at N = 1 and a rank's
# 1/8 share with each, alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r06x_pytest_image.log 2>&1 || exit $?
tail -1 gpurun_out/r06x_pytest_image.log
: > gpurun_out/r06x_bench.jsonl
for rep in 1 2; do
  for rb in torch pt; do
    for s in "" "--share-of 8"; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --readback $rb $s > gpurun_out/r06x_run.log 2>&1 || exit $?
      python3 -c "import json,sys; j=json.loads([l for l in open('gpurun_out/r06x_run.log') if l.startswith('{')][-1]); print(json.dumps({'rep': $rep, 'readback': '$rb', 'share': '$s', 'value': j['value'], 'ms': j['ms_per_step'], 'render_ms': j['roofline'].get('render_ms_steps')}))" | tee -a gpurun_out/r06x_bench.jsonl
    done
  done
done
