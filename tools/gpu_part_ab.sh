#!/bin/bash
# One GPU session for the partition planner (layout.cpp PartRefiner): the
# partitioned-kernel GPU tests at the refined plan, PEG8064 bench lines with and
# without the refinement (same box, interleaved), and WRITE_SIZE passes of
# bp_part_kernel for: the refined plan, the relabelling-only plan, and the
# refined plan without the interior-last column order (plain launches,
# KML_COOP_LAUNCH=0: DESIGN.md W3).  Outputs under gpurun_out/$1/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-part_ab}; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${TESTS_K:-partition or peg8064 or PEG8064 or exact_path or reference_counters or demap or 64qam or 64QAM}" > $O/gpu_tests.log 2>&1 || exit $?
ROUNDS=${ROUNDS:-2} WORKLOADS=peg8064 LIBS="main main:KML_PART_REFINE=0 ${EXTRA_LIBS}" bash tools/gpu_ab.sh ${1:-part_ab} || exit $?
if [ -n "$BG2_LIBS" ]; then
  ROUNDS=${ROUNDS:-2} WORKLOADS=bg2 LIBS="$BG2_LIBS" bash tools/gpu_ab.sh ${1:-part_ab} || exit $?
fi
cd /tmp && export TMPDIR=/tmp
P="--steps 2 --warmup 1 --no-cpu-baseline --no-ber-match --full-loop-batches 0 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096"
for v in refined:KML_PART_REFINE=1 relabel:KML_PART_REFINE=0 nointerior:KML_PART_INTERIOR_LAST=0; do
  tag=${v%%:*}; ev=${v#*:}
  export KML_PART_REFINE=1 KML_PART_INTERIOR_LAST=1 KML_COOP_LAUNCH=0
  export $ev
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/w_$tag -o run --output-format csv -- python3 $R/bench.py $P > $O/w_$tag.log 2>&1 || exit $?
done
unset KML_PART_REFINE KML_PART_INTERIOR_LAST KML_COOP_LAUNCH
for tag in refined relabel nointerior; do
  echo "== $tag" >> $O/summary.txt
  python3 $R/tools/pmc_summary.py $O/w_$tag --kernel bp_part_kernel >> $O/summary.txt 2>&1
  python3 $R/tools/pmc_summary.py $O/w_$tag --kernel demap_kernel >> $O/summary.txt 2>&1
done
cat $O/summary.txt
