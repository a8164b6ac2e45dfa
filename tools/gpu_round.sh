#!/bin/bash
# One GPU session: tests, benches for every BASELINE config, rocprofv3 traces and PMC passes.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/prof $O/pmc_f $O/pmc_w
cd $R
step() { echo "== $1" >> $O/steps.log; }
step tests
timeout -k 10 700 python -m pytest tests/test_gpu_parity.py -q -m gpu -s --maxfail=30 > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
[ $rc -le 1 ] || exit $rc
step bench
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $O/bench.log 2>&1 || exit $?
step bench_blind
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --blind --no-cpu-baseline > $O/bench_blind.log 2>&1 || exit $?
step bench_bg2
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --no-cpu-baseline > $O/bench_bg2.log 2>&1 || exit $?
step bench_peg8064
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --no-cpu-baseline > $O/bench_peg8064.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_bench.log 2>&1 || exit $?
step pmc_fetch
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_f.log 2>&1 || exit $?
step pmc_write
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_w.log 2>&1 || exit $?
step done
