#!/bin/bash
# rocprofv3 kernel traces + PMC passes for the secondary kernels' workloads
# (tools/pmc_workload.sh per workload): PEG8064/64QAM blind (bp_part_kernel,
# km_fused_kernel, cand_metric_kernel, demap), BG2/16QAM known (bp_irregular_kernel),
# PEG2304/QPSK blind (km_fused_kernel, cand_metric_kernel).
set -o pipefail
bash tools/pmc_workload.sh peg8064 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --no-ber-match || exit $?
bash tools/pmc_workload.sh bg2 --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --no-ber-match || exit $?
bash tools/pmc_workload.sh blind2304 --blind --no-ber-match || exit $?
