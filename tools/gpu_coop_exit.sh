#!/bin/bash
# Diagnostic: rocprofv3 --kernel-trace of the PEG8064 bench (cooperative
# launch) with the process's memory map dumped before exit, so the crash at
# exit (W3) can be attributed to a library.  KML_EXIT_RESET=1 (passed through)
# tears the device down with hipDeviceReset before exit().  The traced run is
# the last GPU step.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/coop_exit${KML_EXIT_RESET:+_reset}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
KML_DUMP_MAPS=$O/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ber-match --full-loop-batches 0 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 > $O/t.json 2> $O/t.log
echo "rc=$?" >> $O/t.log
