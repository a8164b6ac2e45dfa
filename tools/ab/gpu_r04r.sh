#!/bin/bash
# Round-4: BG2 irregular plan, seeded within-SIMD orders of its pair and
# single waves (KML_IRR_SEED; 0 = the LPT order): bp_irregular launch time.
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
BG2="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 3"
for s in 0 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18 19 0; do
  KML_LIB=kmldpc_amd/libkmldpc_amd_seed.so KML_IRR_SEED=$s timeout -k 10 200 python bench.py $BG2 $F > $O/bg2_$s.json 2> $O/bg2_$s.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/bg2_$s.json').read().strip().splitlines()[-1]); print('seed $s', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))" | tee -a $O/summary.txt
done
