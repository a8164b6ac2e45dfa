#!/bin/bash
# Quick GPU iteration: every GPU test, then the bench lines named in $BENCHES
# (default: the headline).  Outputs under gpurun_out/$1/.
#   headline  python bench.py (known-H PEG2304, 20 iterations)
#   blind     PEG2304 blind k-means
#   bg2       5G BG2, 50 iterations
#   peg8064   PEG8064 / 64QAM blind
set -o pipefail
O=gpurun_out/${1:-quick}; mkdir -p $O
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1 || exit $?
for b in ${BENCHES:-headline}; do
  case $b in
    headline) A="--no-cpu-baseline" ;;
    headline_cpu) A="" ;;
    blind) A="--blind --no-cpu-baseline" ;;
    bg2) A="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5 --no-cpu-baseline" ;;
    peg8064) A="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 --no-cpu-baseline" ;;
    *) echo "unknown bench $b"; exit 2 ;;
  esac
  timeout -k 10 200 python bench.py $A > $O/bench_$b.json 2> $O/bench_$b.err || exit $?
done
