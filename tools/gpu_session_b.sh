# Round-5 session B: bp_part_kernel split-VN A/B (PEG8064 blind, same box) and
# the partitioned parity tests under the split build.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
PG="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 --no-cpu-baseline"
for r in 1 2; do
timeout -k 10 300 python bench.py $PG > $O/peg_main_$r.json 2>> $O/peg.err || exit $?
KML_LIB=kmldpc_amd/libkmldpc_amd_split.so timeout -k 10 300 python bench.py $PG > $O/peg_split_$r.json 2>> $O/peg.err || exit $?
done
KML_LIB=kmldpc_amd/libkmldpc_amd_split.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "partitioned or peg8064 or PEG8064" > $O/split_tests.log 2>&1 || exit $?
