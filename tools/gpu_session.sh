# Round-5 session A: the k-means / parity GPU tests, the blind bench line with
# its k-means A/B (flagged words by rank vs owned words), k-means phase stamps,
# and the BG2 degree-1 cost-model A/B.  Every GPU step has its own time limit;
# the script stops at the first failure.  Outputs under gpurun_out/r05a/.
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "kmeans or reference_stream or pending_abort or partitioned or golden or screen" > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
timeout -k 10 300 python bench.py --blind --no-cpu-baseline > $O/bench_blind_$r.json 2>> $O/bench_blind.err || exit $?
KML_KM_BAL=0 timeout -k 10 300 python bench.py --blind --no-cpu-baseline > $O/bench_blind_own_$r.json 2>> $O/bench_blind.err || exit $?
done
KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so timeout -k 10 200 python tools/km_stamps.py > $O/km_stamps.txt 2>&1 || exit $?
BG="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5 --no-cpu-baseline"
for r in 1 2; do
timeout -k 10 300 python bench.py $BG > $O/bg2_main_$r.json 2>> $O/bg2.err || exit $?
KML_LIB=kmldpc_amd/libkmldpc_amd_cost1.so timeout -k 10 300 python bench.py $BG > $O/bg2_cost1_$r.json 2>> $O/bg2.err || exit $?
done
