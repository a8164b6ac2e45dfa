set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "kmeans or reference_stream or pending_abort or partitioned or golden or screen" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --blind > $O/bench_blind.json 2> $O/bench_blind.err || exit $?
KML_KM_BAL=0 timeout -k 10 300 python bench.py --blind --no-cpu-baseline > $O/bench_blind_own.json 2>> $O/bench_blind.err || exit $?
KML_KM_HALF=0 timeout -k 10 300 python bench.py --blind --no-cpu-baseline > $O/bench_blind_full.json 2>> $O/bench_blind.err || exit $?
KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so timeout -k 10 200 python tools/km_stamps.py > $O/km_stamps.txt 2>&1 || exit $?
BG="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5"
for r in 1 2; do
timeout -k 10 300 python bench.py $BG > $O/bg2_main_$r.json 2>> $O/bg2.err || exit $?
KML_LIB=kmldpc_amd/libkmldpc_amd_cost1.so timeout -k 10 300 python bench.py $BG > $O/bg2_cost1_$r.json 2>> $O/bg2.err || exit $?
done
# W3: the standalone cooperative-launch program under rocprofv3 (control first, then the cooperative form; last steps)
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/$O/w3_plain -o run --output-format csv -- $R/kmldpc_amd/bin/coop_exit -1 > $R/$O/w3_plain.log 2>&1
rc=$?; echo "rc=$rc" >> $R/$O/w3_plain.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/$O/w3_coop -o run --output-format csv -- $R/kmldpc_amd/bin/coop_exit 1 > $R/$O/w3_coop.log 2>&1
echo "rc=$?" >> $R/$O/w3_coop.log
