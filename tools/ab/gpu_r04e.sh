#!/bin/bash
# Round-4: bp_part2_kernel with prefetched receives.  Partitioned-path GPU
# tests, bench A/B (groups of 8, two slots, vs groups of 4, one slot), and a
# kernel trace of the groups-of-8 chain (dispatch durations).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04e; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "part or 8064 or abort or coop" > $O/gpu_tests.log 2>&1 || exit $?
KML_PART_G=8 KML_PART_MODE=2wg timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "partitioned or peg8064_64qam" > $O/gpu_tests_2wg.log 2>&1 || exit $?
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
for r in 1 2; do
  for cfg in 8:2slot 8:2wg 4:1slot; do
    gsz=${cfg%%:*}; mode=${cfg##*:}
    KML_PART_G=$gsz KML_PART_MODE=$mode timeout -k 10 200 python bench.py $B8064 --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/p8064_${mode}_$r.json 2> $O/p8064_${mode}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/p8064_${mode}_$r.json').read().strip().splitlines()[-1]); print('p8064 $cfg $r', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'), d['roofline'].get('avg_launch_ms'))" >> $O/summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp
KML_PART_G=8 KML_COOP_LAUNCH=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/t8 -o run --output-format csv -- python3 $R/bench.py $B8064 --steps 2 --warmup 1 --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/t8.json 2> $O/t8.log || exit $?
cat $O/summary.txt
