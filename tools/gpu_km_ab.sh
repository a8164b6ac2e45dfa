#!/bin/bash
# A/B of library builds on the blind PEG2304 bench (same box): $LIBS names
# kmldpc_amd/libkmldpc_amd_<x>.so suffixes ("" = the product build).
set -o pipefail
O=gpurun_out/${1:-km_ab}; mkdir -p $O
A="--blind --no-cpu-baseline --no-ber-match --full-loop-batches 0"
for r in 1 2; do
  for l in ${LIBS:-oldkm main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
  done
done
