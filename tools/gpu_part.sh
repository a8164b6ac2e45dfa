#!/bin/bash
# PEG8064 partitioned-kernel check on the GPU box: parity tests for the
# cooperative kernels, bench lines per tiling, phase stamps.  Outputs under
# gpurun_out/$1/.
set -o pipefail
O=gpurun_out/${1:-part}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "8064 or cooperative" > $O/tests_8064.log 2>&1 || exit $?
for T in ${TILES:-1024}; do
  KML_PART=$T timeout -k 10 120 python bench.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --batch 4096 --steps 3 --no-cpu-baseline > $O/bench_part$T.json 2>&1 || exit $?
done
timeout -k 10 120 python tools/part_stamps.py > $O/stamps.txt 2>&1 || exit $?
