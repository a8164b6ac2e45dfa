#!/bin/bash
# k-means iteration: its GPU tests, then the blind bench lines (incremental
# assignment on, then off for A/B).
set -o pipefail
O=gpurun_out/${1:-km}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "kmeans or blind or decode_frames or reference_stream" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --blind --no-cpu-baseline > $O/bench_blind.json 2> $O/bench_blind.err || exit $?
KML_KM_INCR=0 timeout -k 10 200 python bench.py --blind --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/bench_blind_noincr.json 2> $O/bench_blind_noincr.err || exit $?
timeout -k 10 200 python bench.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 --no-cpu-baseline > $O/bench_peg8064.json 2> $O/bench_peg8064.err || exit $?
