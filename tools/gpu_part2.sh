#!/bin/bash
# PEG8064 partitioned kernel: parity tests, then the cfg4 bench line with the
# tagged exchange on and off.  Outputs under gpurun_out/$1/.
set -o pipefail
O=gpurun_out/${1:-part2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "8064 or cooperative or partitioned" > $O/tests_8064.log 2>&1 || exit $?
for T in ${TILES:-1024}; do
  for TG in 1 0; do
    KML_PART=$T KML_PART_TAGGED=$TG timeout -k 10 120 python bench.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --batch 4096 --steps 5 --no-cpu-baseline --no-ber-match > $O/bench_known_T${T}_tg$TG.json 2>&1 || exit $?
    KML_PART=$T KML_PART_TAGGED=$TG timeout -k 10 120 python bench.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 --no-cpu-baseline --no-ber-match > $O/bench_blind_T${T}_tg$TG.json 2>&1 || exit $?
  done
done
