#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-km}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "kmeans or blind or decode_frames or reference_stream" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/km_stamps.py > $O/stamps.txt 2>&1 || exit $?
LIBS="${LIBS:-oldkm main}" bash tools/gpu_km_ab.sh ${1:-km}/ab || exit $?
