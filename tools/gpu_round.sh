#!/bin/bash
# One GPU session for the round's evidence: the GPU tests, bench lines for every
# BASELINE config, a rocprofv3 kernel trace of the headline bench, and PMC passes
# (one counter group per run, no trace domains).  Every GPU step has its own time
# limit; the script stops at the first failure.  Outputs under gpurun_out/round/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
step() { echo "== $1 $(date +%T)" >> $O/steps.log; }
step tests
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
step bench
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
step bench_blind
timeout -k 10 300 python bench.py --blind --no-cpu-baseline > $O/bench_blind.json 2> $O/bench_blind.err || exit $?
step bench_bg2
timeout -k 10 300 python bench.py --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5 --no-cpu-baseline > $O/bench_bg2.json 2> $O/bench_bg2.err || exit $?
step bench_peg8064
timeout -k 10 300 python bench.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 --no-cpu-baseline > $O/bench_peg8064.json 2> $O/bench_peg8064.err || exit $?
cd /tmp && export TMPDIR=/tmp
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || exit $?
P="--steps 2 --warmup 1 --no-cpu-baseline"
step pmc_fetch
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py $P > $O/pmc_fetch.log 2>&1 || exit $?
step pmc_write
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py $P > $O/pmc_write.log 2>&1 || exit $?
step pmc_a
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pmc_a -o run --output-format csv -- python3 $R/bench.py $P > $O/pmc_a.log 2>&1 || exit $?
step pmc_b
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/pmc_b -o run --output-format csv -- python3 $R/bench.py $P > $O/pmc_b.log 2>&1 || exit $?
step pmc_c
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS SQ_INSTS_VALU_FLOPS_FP64 -d $O/pmc_c -o run --output-format csv -- python3 $R/bench.py $P > $O/pmc_c.log 2>&1 || exit $?
step done
