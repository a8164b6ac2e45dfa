set -o pipefail
O=gpurun_out/st6; mkdir -p $O
L=$(pwd)/kmldpc_amd
KML_LIB=$L/libkmldpc_amd_stamps.so timeout -k 10 120 python tools/km_stamps.py > $O/km_qpsk_weak.txt 2>&1 || exit $?
KML_LIB=$L/libkmldpc_amd_stampsnoweak.so timeout -k 10 120 python tools/km_stamps.py > $O/km_qpsk_noweak.txt 2>&1 || exit $?
MATRIX=PEG8064regular0.5.txt MODEM=6bits_64QAM_Gray.txt SNR=6.77 B=4096 KML_LIB=$L/libkmldpc_amd_stamps.so timeout -k 10 120 python tools/km_stamps.py > $O/km_64qam_weak.txt 2>&1 || exit $?
MATRIX=PEG8064regular0.5.txt MODEM=6bits_64QAM_Gray.txt SNR=6.77 B=4096 KML_LIB=$L/libkmldpc_amd_stampsnoweak.so timeout -k 10 120 python tools/km_stamps.py > $O/km_64qam_noweak.txt 2>&1 || exit $?
KML_PART_TAGGED=1 KML_LIB=$L/libkmldpc_amd_stamps.so timeout -k 10 150 python tools/part_stamps.py > $O/part_tagged.txt 2>&1 || exit $?
KML_PART_REFINE=0 KML_PART_TAGGED=1 KML_LIB=$L/libkmldpc_amd_stamps.so timeout -k 10 150 python tools/part_stamps.py > $O/part_tagged_relabel.txt 2>&1 || exit $?
tail -n 30 $O/*.txt
