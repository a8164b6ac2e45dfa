#!/bin/bash
# Headline bench lines only (bp_regular_kernel) for $LIBS (kmldpc_amd/libkmldpc_amd_<x>.so, "main" = product).
set -o pipefail
O=gpurun_out/${1:-reg_bench}; mkdir -p $O
A="--no-cpu-baseline --no-ber-match --full-loop-batches 0 --steps 20"
for r in 1 2; do
  for l in ${LIBS:-main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
  done
done
