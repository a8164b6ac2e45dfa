#!/bin/bash
# Same-box check of the bench lines against rocprofv3: each workload's bench
# line, then `rocprofv3 --kernel-trace --stats` of the identical command on the
# same box (the traced partitioned kernel with plain launches under the
# profiler: KML_COOP_LAUNCH=0, same residency; the bench line itself with the
# shipped cooperative launch).  Outputs gpurun_out/samebox/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/samebox; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, coop env, bench args...
  local n=$1 env=$2; shift 2
  echo "== $n $(date +%T)" >> $O/steps.log
  timeout -k 10 300 python3 $R/bench.py "$@" > $O/$n.json 2> $O/$n.err || return $?
  env $env timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$n -o run --output-format csv -- python3 $R/bench.py "$@" > $O/$n.traced.json 2> $O/$n.traced.log || return $?
}
run headline KML_COOP_LAUNCH=1 || exit $?
run blind KML_COOP_LAUNCH=1 --blind || exit $?
run bg2 KML_COOP_LAUNCH=1 --matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5 || exit $?
run peg8064 KML_COOP_LAUNCH=0 --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 || exit $?
echo "== done $(date +%T)" >> $O/steps.log
