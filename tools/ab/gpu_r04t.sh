#!/bin/bash
# Round-4: k-means ordered-sum scan with 4 / 6 elements per lane and step
# (p4, p6) vs 5 (main); blind PEG2304 QPSK.
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
for r in 1 2; do
  for l in main p4 p6; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py --blind --steps 3 $F > $O/blind_${l}_$r.json 2> $O/blind_${l}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/blind_${l}_$r.json').read().strip().splitlines()[-1]); print('blind $l $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" | tee -a $O/summary.txt
  done
done
