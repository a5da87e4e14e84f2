#!/bin/bash
# Round 5: the leaf pass's own chunking (16 entries) beside the traversal's (8): leaf-pass parity
# variants, the boat / CornellBox2 bands, and in process against ablib/chunk16 (16 for both) on the
# boat and on CornellBox2 with every mesh.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05y_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05y_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_config_bands.py tests/test_gpu_fast_trees.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > $P/r05y_pytest_bands.log 2>&1
rc=$?; tail -2 $P/r05y_pytest_bands.log; [ $rc -eq 0 ] || exit $rc
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
: > $P/r05y_ab_passchunks.log
for args in "--scene MedievalBoat --res 960 --spp 8 --depth 16" "--scene CornellBox2 --all-meshes --res 1024 --spp 4 --depth 16"; do
  timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/chunk16/libpt_hip.so $args --rounds 3 >> $P/r05y_ab_passchunks.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 $P/r05y_ab_passchunks.log; exit $rc; }
  timeout -k 10 600 python3 scripts/ab_libs.py ablib/chunk16/libpt_hip.so $L $args --rounds 3 >> $P/r05y_ab_passchunks.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 $P/r05y_ab_passchunks.log; exit $rc; }
done
grep '"lib"' $P/r05y_ab_passchunks.log
