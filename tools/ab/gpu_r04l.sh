#!/bin/bash
# Round-4: metric kernel with the candidates' hard bits packed per column
# (main) vs HEAD (prev); QPSK metric at >= 6 / 8 waves per SIMD (w6, w8).
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "metric or demap or blind or candidates or adversarial or histogram" > $O/gpu_tests.log 2>&1 || exit $?
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
for r in 1 2; do
  for l in main prev w6 w8; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py --blind --steps 3 $F > $O/blind_${l}_$r.json 2> $O/blind_${l}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/blind_${l}_$r.json').read().strip().splitlines()[-1]); print('blind $l $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" >> $O/summary.txt
    if [ "$l" = main ] || [ "$l" = prev ]; then
      KML_LIB=$L timeout -k 10 200 python bench.py $B8064 $F > $O/p8064_${l}_$r.json 2> $O/p8064_${l}_$r.err || exit $?
      python3 -c "import json; d=json.loads(open('$O/p8064_${l}_$r.json').read().strip().splitlines()[-1]); print('p8064 $l $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" >> $O/summary.txt
    fi
  done
done
cat $O/summary.txt
