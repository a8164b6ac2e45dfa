set -o pipefail
KML_LIB=$(pwd)/kmldpc_amd/libkmldpc_amd_base.so bash tools/pmc_workload.sh headline_base || exit $?
bash tools/pmc_workload.sh headline || exit $?
bash tools/pmc_workload.sh peg8064 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 || exit $?
