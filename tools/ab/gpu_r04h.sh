#!/bin/bash
# Round-4: the metric screen in log2 units without clip / normalisation
# (cand_metric_kernel): demap / metric / blind tests, then the blind benches.
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "metric or demap or blind or candidates or adversarial" > $O/gpu_tests.log 2>&1 || exit $?
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
for r in 1 2; do
  timeout -k 10 200 python bench.py $B8064 --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/p8064_$r.json 2> $O/p8064_$r.err || exit $?
  timeout -k 10 200 python bench.py --blind --steps 3 --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/blind_$r.json 2> $O/blind_$r.err || exit $?
  for w in p8064 blind; do
    python3 -c "import json; d=json.loads(open('$O/${w}_$r.json').read().strip().splitlines()[-1]); print('$w $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" >> $O/summary.txt
  done
done
cat $O/summary.txt
