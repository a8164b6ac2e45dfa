set -o pipefail
O=gpurun_out/km13; mkdir -p $O
timeout -k 10 120 python tools/km_stamps.py > $O/stamps.txt 2>&1 || exit $?
bash tools/pmc_workload.sh blind2304_km13 --blind --no-ber-match --full-loop-batches 0 || exit $?
