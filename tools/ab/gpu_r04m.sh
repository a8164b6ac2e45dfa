#!/bin/bash
# Round-4: the QPSK metric at 8 waves per SIMD as the default (main); the
# 64QAM metric at 4 waves per SIMD (b4) vs 3 (main).
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "metric or demap or blind or candidates or adversarial or histogram" > $O/gpu_tests.log 2>&1 || exit $?
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
for r in 1 2; do
  timeout -k 10 200 python bench.py --blind --steps 3 $F > $O/blind_main_$r.json 2> $O/blind_main_$r.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/blind_main_$r.json').read().strip().splitlines()[-1]); print('blind main $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" >> $O/summary.txt
  for l in main b4; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py $B8064 $F > $O/p8064_${l}_$r.json 2> $O/p8064_${l}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/p8064_${l}_$r.json').read().strip().splitlines()[-1]); print('p8064 $l $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" >> $O/summary.txt
  done
done
cat $O/summary.txt
