#!/bin/bash
# Round-4: bp_part tagged kernel with its receive lists in LDS (main) vs in
# registers (prev: the c2v list spilled); partitioned tests first.
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "partitioned or peg8064 or abort" > $O/gpu_tests.log 2>&1 || exit $?
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
for r in 1 2 3; do
  for l in main prev; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py $B8064 $F > $O/p8064_${l}_$r.json 2> $O/p8064_${l}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/p8064_${l}_$r.json').read().strip().splitlines()[-1]); print('p8064 $l $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'), d['roofline'].get('avg_launch_ms'))" >> $O/summary.txt
  done
done
cat $O/summary.txt
