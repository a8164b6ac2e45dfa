set -o pipefail
O=gpurun_out/ab1; mkdir -p $O
for v in ${VARIANTS}; do
  KML_LIB=$PWD/kmldpc_amd/ab/$v.so timeout -k 10 120 python bench.py --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5 --no-cpu-baseline > $O/$v.json 2>$O/$v.err || exit $?
done
