#!/bin/bash
# GPU tests, then A/B of library builds on the PEG8064 blind bench (same box):
# $LIBS names kmldpc_amd/libkmldpc_amd_<x>.so suffixes ("main" = the product build).
set -o pipefail
O=gpurun_out/${1:-part_ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/part_stamps.py > $O/stamps.txt 2>&1 || exit $?
A="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 5 --no-cpu-baseline --no-ber-match --full-loop-batches 0"
for r in 1 2; do
  for l in ${LIBS:-prev main}; do
    if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
    KML_LIB=$L timeout -k 10 200 python bench.py $A > $O/${l}_$r.json 2> $O/${l}_$r.err || exit $?
  done
done
