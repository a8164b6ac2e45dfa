#!/bin/bash
# One GPU session for the round's evidence when boxes are scarce: the PMC passes
# of $PMC_WORKLOADS (default: headline), their summary merged into the box copy's
# profiles/pmc_bp.json (tools/collect_round.py --pmc, so the bench lines carry
# the counter views), then tools/gpu_round.sh (GPU tests + the four bench
# lines), then an A/B of the headline against $AB_LIBS builds.  Every GPU step
# has its own time limit and the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
echo "== pmc $(date +%T)" >> gpurun_out/final_steps.log
WORKLOADS="${PMC_WORKLOADS:-headline}" bash tools/gpu_pmc_all.sh || exit $?
python3 tools/collect_round.py ${PRE:-r03_v2} --pmc > gpurun_out/collect_box.log 2>&1 || exit $?
echo "== round $(date +%T)" >> gpurun_out/final_steps.log
bash tools/gpu_round.sh || exit $?
if [ -n "$AB_LIBS" ]; then
  echo "== ab $(date +%T)" >> gpurun_out/final_steps.log
  ROUNDS=1 LIBS="$AB_LIBS" WORKLOADS="${AB_WORKLOADS:-headline}" bash tools/gpu_ab.sh ab_final || exit $?
fi
echo "== done $(date +%T)" >> gpurun_out/final_steps.log
