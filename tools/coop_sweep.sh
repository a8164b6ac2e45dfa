#!/bin/bash
# A/B of the cooperative BP kernel's tilings on PEG8064 (KML_COOP=G,T).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "peg8064" > gpurun_out/gt8064.log 2>&1 || exit $?
for cfg in 4,512 4,1024 8,512 8,1024; do
  KML_COOP=$cfg timeout -k 10 120 python bench.py --no-cpu-baseline --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --batch 4096 --steps 3 > gpurun_out/coop_${cfg/,/_}.log 2>&1 || exit $?
done
