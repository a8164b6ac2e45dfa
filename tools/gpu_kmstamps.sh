#!/bin/bash
# k-means and partitioned-BP phase stamps (needs `make stamps`); outputs gpurun_out/$1/.
set -o pipefail
O=gpurun_out/${1:-st}; mkdir -p $O
export KML_LIB=$(pwd)/kmldpc_amd/libkmldpc_amd_stamps.so
timeout -k 10 120 python tools/km_stamps.py > $O/km_qpsk.txt 2>&1 || exit $?
KML_PART_TAGGED=1 timeout -k 10 120 python tools/part_stamps.py > $O/part_tagged.txt 2>&1 || exit $?
