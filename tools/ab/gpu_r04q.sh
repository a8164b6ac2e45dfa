#!/bin/bash
# Round-4: bp_regular VN-phase wave priorities: falling levels (main) vs by
# wave age until the last column (a2) / for the whole phase (a3); headline.
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
F="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
for r in 1 2 3; do
  for l in main a2 a3; do
    L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
    KML_LIB=$L timeout -k 10 200 python bench.py --steps 5 $F > $O/head_${l}_$r.json 2> $O/head_${l}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/head_${l}_$r.json').read().strip().splitlines()[-1]); print('headline $l $r', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))" >> $O/summary.txt
  done
done
cat $O/summary.txt
