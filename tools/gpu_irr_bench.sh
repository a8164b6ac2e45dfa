#!/bin/bash
# BG2 bench lines only (bp_irregular_kernel) for $LIBS (kmldpc_amd/libkmldpc_amd_<x>.so, "main" = product).
set -o pipefail
O=gpurun_out/${1:-irr_bench}; mkdir -p $O
A="--no-cpu-baseline --no-ber-match --full-loop-batches 0 --steps 20 --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384"
for r in 1 2; do
  for l in ${LIBS:-main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
  done
done
