#!/bin/bash
# Round-4: phase stamps of the BG2 irregular kernel, the headline regular
# kernel and the k-means (stamps build) at the current sources.
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
export KML_LIB=$(pwd)/kmldpc_amd/libkmldpc_amd_stamps.so
timeout -k 10 180 python tools/irr_stamps.py > $O/irr.txt 2>&1 || exit $?
timeout -k 10 180 python tools/reg_stamps.py > $O/reg.txt 2>&1 || exit $?
timeout -k 10 180 python tools/km_stamps.py > $O/km.txt 2>&1 || exit $?
