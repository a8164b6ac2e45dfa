#!/bin/bash
# Headline A/B of library builds (same box): GPU parity tests of the BP paths,
# stamps, then bench lines; $LIBS: kmldpc_amd/libkmldpc_amd_<x>.so ("main" = product),
# $BENCH_ARGS: extra bench.py arguments (another workload), $NOSTAMPS=1 skips the stamps.
set -o pipefail
O=gpurun_out/${1:-reg_ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bp or decode or reference or fused or demap or driver or bench" > $O/gpu_tests.log 2>&1 || exit $?
[ -n "$NOSTAMPS" ] || timeout -k 10 120 python tools/reg_stamps.py > $O/stamps.txt 2>&1 || exit $?
A="--no-cpu-baseline --no-ber-match --full-loop-batches 0 --steps 20 $BENCH_ARGS"
for r in 1 2; do
  for l in ${LIBS:-prev main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
  done
done
