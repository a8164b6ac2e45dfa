#!/bin/bash
# One GPU session of round-6 A/Bs: the GPU tests (filter $TESTS_K, all when
# empty), then same-box bench lines per workload (tools/gpu_ab.sh, $ROUNDS
# rounds interleaved) for the library sets $AB_<workload> (e.g.
# AB_peg8064="main main:KML_PART_REFINE=0 base"), then optional WRITE_SIZE
# passes of the PEG8064 workload ($PMC_W=1: refined / relabel-only /
# no interior-last plans, plain launches KML_COOP_LAUNCH=0: DESIGN.md W3), and
# the k-means stamps ($KMSTAMPS=1).  Outputs under gpurun_out/$1/; every GPU
# step under its own limit, the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-r06ab}
O=$R/gpurun_out/$N; mkdir -p $O
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1 || exit $?
fi
for w in headline blind bg2 peg8064; do
  v=AB_$w
  if [ -n "${!v}" ]; then
    ROUNDS=${ROUNDS:-2} WORKLOADS=$w LIBS="${!v}" bash tools/gpu_ab.sh $N > /dev/null || exit $?
  fi
done
if [ "${KMSTAMPS:-0}" = 1 ]; then
  timeout -k 10 120 python tools/km_stamps.py > $O/km_stamps.txt 2>&1 || exit $?
fi
if [ "${PMC_W:-0}" = 1 ]; then
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
fi
cat $O/summary.txt
