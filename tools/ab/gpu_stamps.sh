#!/bin/bash
# Phase stamps of the partitioned kernel, tagged and barrier exchange (needs `make stamps`).
set -o pipefail
O=gpurun_out/${1:-st}; mkdir -p $O
KML_PART_TAGGED=1 timeout -k 10 120 python tools/part_stamps.py > $O/tagged.txt 2>&1 || exit $?
KML_PART_TAGGED=0 timeout -k 10 120 python tools/part_stamps.py > $O/legacy.txt 2>&1 || exit $?
