#!/bin/bash
# k-means A/B on one box: the k-means GPU parity tests, km stamps of the
# product build, then blind PEG2304 bench lines for $LIBS (kmldpc_amd/libkmldpc_amd_<x>.so, "main" = product).
set -o pipefail
O=gpurun_out/${1:-km_ab2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "kmeans or blind or metric or candidate" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/km_stamps.py > $O/stamps.txt 2>&1 || exit $?
A="--blind --no-cpu-baseline --no-ber-match --full-loop-batches 0"
for r in 1 2; do
  for l in ${LIBS:-prev main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
  done
done
