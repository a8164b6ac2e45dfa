#!/bin/bash
# A/B of library builds on one box for the headline (bp_regular) and BG2
# (bp_irregular) workloads: GPU parity tests of the BP paths, both kernels'
# stamps, then bench lines for $LIBS (kmldpc_amd/libkmldpc_amd_<x>.so, "main" = product).
set -o pipefail
O=gpurun_out/${1:-ab_both}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bp or decode or reference or fused or demap or driver or bench" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/reg_stamps.py > $O/reg_stamps.txt 2>&1 || exit $?
timeout -k 10 120 python tools/irr_stamps.py > $O/irr_stamps.txt 2>&1 || exit $?
A="--no-cpu-baseline --no-ber-match --full-loop-batches 0 --steps 20"
G="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384"
for r in 1 2; do
  for l in ${LIBS:-prev main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
    KML_LIB=$L timeout -k 10 200 python bench.py $A $G > $O/bg2_${l}_$r.json 2> $O/bg2_${l}_$r.err || exit $?
  done
done
