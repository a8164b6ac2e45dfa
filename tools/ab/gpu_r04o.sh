#!/bin/bash
# Round-4: BG2 irregular plan with the heaviest pair wave of a SIMD sharing its
# lane wave with the lightest single wave (main) vs HEAD (prev); stamps.
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bg2 or irregular or 5g or g2" > $O/gpu_tests.log 2>&1 || exit $?
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
BG2="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5"
for r in 1 2 3; do
  for l in main prev; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py $BG2 $F > $O/bg2_${l}_$r.json 2> $O/bg2_${l}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/bg2_${l}_$r.json').read().strip().splitlines()[-1]); print('bg2 $l $r', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))" >> $O/summary.txt
  done
done
KML_LIB=$(pwd)/kmldpc_amd/libkmldpc_amd_stamps.so timeout -k 10 180 python tools/irr_stamps.py > $O/irr.txt 2>&1 || exit $?
cat $O/summary.txt
