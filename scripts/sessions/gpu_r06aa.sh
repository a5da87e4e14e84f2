#!/bin/bash
# Round 6: batch k's accumulation on its own stream beside batch k + 1 (double radiance buffer):
# parity of the multi-batch renders, in-process A/B against HEAD (H), the bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "batch or accum or profile or wavefront_default or multi or part" --timeout 500 --timeout-method thread > gpurun_out/r06aa_parity.log 2>&1 || exit $?
tail -1 gpurun_out/r06aa_parity.log
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
H=ablib/head/libpt_hip.so
timeout -k 10 400 python -u scripts/ab_libs.py $H $L $H $L --rounds 3 --async-torch --scene CornellBox --res 1024 --spp 256 --depth 8 > gpurun_out/r06aa_ab_n1.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/ab_libs.py $H $L --rounds 3 --async-torch --scene CornellBox-Glossy --res 1024 --spp 128 --depth 16 > gpurun_out/r06aa_ab_glossy.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06aa_ab_*.log
: > gpurun_out/r06aa_bench.jsonl
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06aa_run.log 2>&1 || exit $?
  python3 -c "import json,sys; j=json.loads([l for l in open('gpurun_out/r06aa_run.log') if l.startswith('{')][-1]); print(json.dumps({'rep': $rep, 'value': j['value'], 'ms': j['ms_per_step']}))" | tee -a gpurun_out/r06aa_bench.jsonl
done
