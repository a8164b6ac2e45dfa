#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-km}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "kmeans or blind or decode_frames or reference_stream" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/km_stamps.py > $O/stamps.txt 2>&1 || exit $?
KML_KM_SCAN=0 timeout -k 10 120 python tools/km_stamps.py > $O/stamps_noscan.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --blind --no-cpu-baseline --full-loop-batches 0 > $O/bench_blind.json 2> $O/bench_blind.err || exit $?
KML_KM_SCAN=0 timeout -k 10 200 python bench.py --blind --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/bench_blind_noscan.json 2> $O/bench_blind_noscan.err || exit $?
