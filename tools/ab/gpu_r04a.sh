#!/bin/bash
# Round-4 first session: the GPU tests, the headline bench line, and the
# PEG8064 kernel trace + PMC passes at HEAD's sources.  The PMC passes launch
# the partitioned kernel plainly (KML_COOP_LAUNCH=0: same occupancy check,
# same residency; a cooperative launch under rocprofv3 crashes the process in
# the runtime's exit teardown, profiles/r03_coop_exit_crash.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04a; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
KML_COOP_LAUNCH=0 WORKLOADS=peg8064 bash tools/gpu_pmc_all.sh || exit $?
