#!/bin/bash
# Round-4: the two-slot partitioned kernel (bp_part2_kernel, groups of 8).
# GPU tests of the partitioned / PEG8064 paths, then bench A/B against the
# one-slot kernel (KML_PART_G=4), two rounds.
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "part or 8064 or integration or exact_path or reference_stream or abort or coop or empty or extreme" > $O/gpu_tests.log 2>&1 || exit $?
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
for r in 1 2; do
  for gsz in 8 4; do
    KML_PART_G=$gsz timeout -k 10 200 python bench.py $B8064 --no-cpu-baseline --full-loop-batches 0 > $O/p8064_g${gsz}_$r.json 2> $O/p8064_g${gsz}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/p8064_g${gsz}_$r.json').read().strip().splitlines()[-1]); print('p8064 G=$gsz $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'), d.get('ber_match'))" >> $O/summary.txt
  done
done
cat $O/summary.txt
