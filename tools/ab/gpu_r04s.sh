#!/bin/bash
# Round-4: FAST demapper with one ProbClip and the unweighted sum (main) vs
# HEAD (prev): demap / metric / fused-demap tests, then PEG8064 blind, BG2 and
# the headline.
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "demap or metric or fused or adversarial or golden or known or exact" > $O/gpu_tests.log 2>&1 || exit $?
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
BG2="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 3"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'), d['roofline'].get('avg_launch_ms'))" >> $O/summary.txt; }
for r in 1 2; do
  for l in main prev; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py $B8064 $F > $O/p8064_${l}_$r.json 2> $O/p8064_${l}_$r.err || exit $?
    line $O/p8064_${l}_$r.json "p8064 $l $r"
    KML_LIB=$L timeout -k 10 200 python bench.py $BG2 $F > $O/bg2_${l}_$r.json 2> $O/bg2_${l}_$r.err || exit $?
    line $O/bg2_${l}_$r.json "bg2 $l $r"
    KML_LIB=$L timeout -k 10 200 python bench.py --steps 5 $F > $O/head_${l}_$r.json 2> $O/head_${l}_$r.err || exit $?
    line $O/head_${l}_$r.json "headline $l $r"
  done
done
cat $O/summary.txt
