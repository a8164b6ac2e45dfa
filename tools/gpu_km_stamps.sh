#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-km_st}; mkdir -p $O
timeout -k 10 120 python tools/km_stamps.py > $O/stamps.txt 2>&1 || exit $?
KML_KM_INCR=0 timeout -k 10 120 python tools/km_stamps.py > $O/stamps_noincr.txt 2>&1 || exit $?
