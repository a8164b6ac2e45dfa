#!/bin/bash
# FAST-division diagnostics on the GPU box (tools/div_stats.py) for the bench
# workloads; outputs gpurun_out/$1/divstats_<w>.json.
set -o pipefail
O=gpurun_out/${1:-divstats}; mkdir -p $O
export KML_LIB=kmldpc_amd/libkmldpc_amd_divstats.so
timeout -k 10 120 python tools/div_stats.py --batch 4096 --out $O/divstats_headline.json > /dev/null || exit $?
timeout -k 10 120 python tools/div_stats.py --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 4096 --out $O/divstats_bg2.json > /dev/null || exit $?
timeout -k 10 180 python tools/div_stats.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 1024 --out $O/divstats_peg8064.json > /dev/null || exit $?
