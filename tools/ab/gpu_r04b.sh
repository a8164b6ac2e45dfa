#!/bin/bash
# Round-4 A/B session: GPU tests of the changed kernels (partitioned BP with
# branch-free tagged stores, k-means scan cache), then bench lines of: base
# (HEAD before these changes) vs main, kmcap3 (k-means list capacity S/3: 8
# codewords per CU?), noproof (the FAST VN division proof's price, measurement
# only), and the k-means / partitioned-BP phase stamps.
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "part or 8064 or kmeans or integration or exact_path or reference_stream or abort or coop" > $O/gpu_tests.log 2>&1 || exit $?
B8064="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"
BBG2="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5"
run() {  # name lib args...
  local n=$1 l=$2; shift 2
  local L=kmldpc_amd/libkmldpc_amd.so; [ "$l" = main ] || L=kmldpc_amd/libkmldpc_amd_$l.so
  KML_KM_OCC=1 KML_LIB=$L timeout -k 10 200 python bench.py "$@" --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/${n}_$l.json 2> $O/${n}_$l.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/${n}_$l.json').read().strip().splitlines()[-1]); print('$n $l', d['value'], d['ms_per_step'], d['stats'].get('stage_ms_per_step'))" >> $O/summary.txt
}
for r in 1 2; do
  run p8064_$r base $B8064
  run p8064_$r main $B8064
  run p8064_$r noanneal $B8064
  run blind$r base --blind
  run blind$r main --blind
  run blind$r kmcap3 --blind
  run head$r main
  run head$r noproof
  run bg2$r main $BBG2
  run bg2$r noproof $BBG2
  run bg2$r irrdefer $BBG2
done
run p8064_3 noproof $B8064
bash tools/gpu_kmstamps.sh r04b_st || exit $?
cat $O/summary.txt
