#!/bin/bash
# The round's PMC evidence: tools/pmc_workload.sh for the four bench workloads
# (headline PEG2304/QPSK known, PEG2304/QPSK blind, BG2/16QAM known,
# PEG8064/64QAM blind).  WORKLOADS selects a subset.
set -o pipefail
for w in ${WORKLOADS:-headline blind bg2 peg8064}; do
  case $w in
    headline) bash tools/pmc_workload.sh headline || exit $? ;;
    blind) bash tools/pmc_workload.sh blind --blind || exit $? ;;
    bg2) bash tools/pmc_workload.sh bg2 --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 || exit $? ;;
    peg8064) bash tools/pmc_workload.sh peg8064 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 || exit $? ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
done
