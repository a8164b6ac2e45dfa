#!/bin/bash
# Round-4 evidence at HEAD: every GPU test, the four bench lines, and the
# kernel traces + PMC passes of every workload (plain launches for the
# partitioned kernel: KML_COOP_LAUNCH=0, same residency; see gpu_r04a.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round; mkdir -p $O
cd $R
step() { echo "== $1 $(date +%T)" >> $O/steps.log; }
step tests
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
step bench
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
step bench_blind
timeout -k 10 300 python bench.py --blind > $O/bench_blind.json 2> $O/bench_blind.err || exit $?
step bench_bg2
timeout -k 10 300 python bench.py --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5 > $O/bench_bg2.json 2> $O/bench_bg2.err || exit $?
step bench_peg8064
timeout -k 10 400 python bench.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 > $O/bench_peg8064.json 2> $O/bench_peg8064.err || exit $?
step pmc
KML_COOP_LAUNCH=0 bash tools/gpu_pmc_all.sh || exit $?
step pmc_done
# the 64QAM demap with the bank-private exp table (variant build): its LDS counters
step pmc_banked
KML_LIB=$R/kmldpc_amd/libkmldpc_amd_banked.so timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_banked/b -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ber-match --full-loop-batches 0 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 > $R/gpurun_out/pmc_banked.log 2>&1 || exit $?
step done2
