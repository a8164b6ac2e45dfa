#!/bin/bash
# Round-4: bp_regular epilogue from the LDS info positions (main) vs global
# reg_pos loads (prev); the fused demap off; bp_part tilings T = 768 / 1024.
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "regular or fused or headline or known" > $O/gpu_tests.log 2>&1 || exit $?
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$2', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'), r.get('avg_launch_ms'))" >> $O/summary.txt; }
for r in 1 2 3; do
  for l in main prev; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py --steps 5 $F > $O/head_${l}_$r.json 2> $O/head_${l}_$r.err || exit $?
    line $O/head_${l}_$r.json "headline $l $r"
  done
done
KML_FUSED_DEMAP=0 timeout -k 10 200 python bench.py --steps 5 $F > $O/head_unfused.json 2> $O/head_unfused.err || exit $?
line $O/head_unfused.json "headline unfused-demap"
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
for t in 512 768 1024; do
  KML_PART=$t timeout -k 10 200 python bench.py $B8064 $F > $O/p8064_$t.json 2> $O/p8064_$t.err || exit $?
  line $O/p8064_$t.json "p8064 T=$t"
done
cat $O/summary.txt
