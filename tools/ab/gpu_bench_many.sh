#!/bin/bash
# Bench lines of several library builds on one box for one workload:
# $LIBS (kmldpc_amd/libkmldpc_amd_<x>.so, "main" = product), $BENCH_ARGS the workload.
set -o pipefail
O=gpurun_out/${1:-bench_many}; mkdir -p $O
A="--no-cpu-baseline --no-ber-match --full-loop-batches 0 $BENCH_ARGS"
for r in 1 2; do
  for l in ${LIBS:-main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
  done
done
