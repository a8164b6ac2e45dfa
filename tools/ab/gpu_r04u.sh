#!/bin/bash
# Round-4: demap_kernel occupancy: 64QAM at 3 waves per SIMD and 16QAM at 4
# (d) vs 2 and unconstrained (main); demap tests with the variant first.
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
KML_LIB=$(pwd)/kmldpc_amd/libkmldpc_amd_d.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "demap or adversarial or golden" > $O/gpu_tests.log 2>&1 || exit $?
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
BG2="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 3"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" | tee -a $O/summary.txt; }
for r in 1 2; do
  for l in main d; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py $B8064 $F > $O/p8064_${l}_$r.json 2> $O/p8064_${l}_$r.err || exit $?
    line $O/p8064_${l}_$r.json "p8064 $l $r"
    KML_LIB=$L timeout -k 10 200 python bench.py $BG2 $F > $O/bg2_${l}_$r.json 2> $O/bg2_${l}_$r.err || exit $?
    line $O/bg2_${l}_$r.json "bg2 $l $r"
  done
done
